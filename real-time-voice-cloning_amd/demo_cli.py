"""End-to-end voice cloning on MI355X: GE2E encoder + Tacotron (PyTorch-ROCm) feeding the HIP
WaveRNN vocoder (BASELINE.json configs[4]; reference ``demo_cli.py:80-217``).

Flow per utterance, as the reference's demo: reference wav -> ``encoder.preprocess_wav`` ->
``encoder.embed_utterance`` -> ``synthesizer.synthesize_spectrograms([text], [embed])`` ->
``vocoder.infer_waveform(spec)`` -> pad 1 s, ``encoder.preprocess_wav`` -> wav file.

Multi-GPU: launched with ``torchrun --nproc-per-node N``, rank r takes utterances r, r + N, ...
(utterances are independent; no collective on the data path), synthesizes its texts as one
Tacotron batch and vocodes its mels as one batch of fold rows (``WaveRNN.generate_batch``);
rank 0 prints one JSON line with the max-over-ranks stage times.

No checkpoints or sample audio exist offline: ``--random-weights SEED`` builds seeded stand-in
weights for the three models (the Tacotron stop-token bias is pinned low, so every utterance
runs ``--max-frames`` decoder steps), and without ``--ref-wav`` a seeded synthetic voiced signal
is the reference utterance. Checkpoints load with ``torch.load(..., weights_only=True)``.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

TEXTS = [
    "Welcome to the voice cloning demonstration running on an accelerator.",
    "The vocoder turns each spectrogram frame into two hundred audio samples.",
    "Every fold of the spectrogram is generated in parallel and cross faded.",
    "This sentence was synthesized with the speaker embedding of the reference.",
    "Recurrent networks are sequential, so latency matters more than bandwidth.",
    "Eight utterances are spread over the devices of one node.",
    "The quick brown fox jumps over the lazy dog.",
    "Thank you for listening to this synthetic voice.",
]


def synthetic_voice(seconds=3.0, sr=16000, seed=0):
    """Seeded voiced signal: a gliding harmonic source with vibrato, formant-ish weights, noise."""
    rng = np.random.default_rng(seed)
    t = np.arange(int(seconds * sr)) / sr
    f0 = 120 + 30 * np.sin(2 * np.pi * 0.7 * t) + 5 * np.sin(2 * np.pi * 5.5 * t)
    phase = 2 * np.pi * np.cumsum(f0) / sr
    wav = sum((1.0 / k) * np.sin(k * phase + rng.uniform(0, 2 * np.pi)) for k in range(1, 25))
    env = 0.6 + 0.4 * np.sin(2 * np.pi * 2.1 * t) ** 2
    wav = env * wav + 0.01 * rng.normal(size=t.size)
    return (0.3 * wav / np.abs(wav).max()).astype(np.float32)


def main():
    ap = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    ap.add_argument("-e", "--enc_model_fpath", default="encoder/saved_models/pretrained.pt")
    ap.add_argument("-s", "--syn_model_fpath", default="synthesizer/saved_models/pretrained/pretrained.pt")
    ap.add_argument("-v", "--voc_model_fpath", default="vocoder/saved_models/pretrained/pretrained.pt")
    ap.add_argument("--random-weights", type=int, default=None,
                    help="seeded stand-in weights for all three models (no checkpoints offline)")
    ap.add_argument("--ref-wav", default=None, help="reference utterance (16-bit / float WAV)")
    ap.add_argument("--utterances", type=int, default=8)
    ap.add_argument("--max-frames", type=int, default=400, help="Tacotron decoder steps cap")
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--out-dir", default=None, help="write demo_output_XX.wav files here")
    ap.add_argument("--vocoder-type", default="fatchord-wavernn")
    ap.add_argument("--repeat", type=int, default=2,
                    help="timed passes over the same utterances; the last one is reported")
    ap.add_argument("--dump", default=None,
                    help="write rank 0's first utterance as the vocoder saw it (normalised mel, "
                         "fold-row labels, seed, noise stream) to this .npz: the GPU parity check of "
                         "the end-to-end run against the oracle (tests/test_gpu_e2e.py)")
    ap.add_argument("--warmup", type=int, default=1,
                    help="untimed passes of a short utterance through the three models first "
                         "(library and kernel initialisation), as a serving process would")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        raise RuntimeError("the MI355X vocoder needs a GPU")
    red_dev = dev  # device of the timing reductions
    if world > 1:  # RCCL with one GPU per rank; gloo when ranks share a GPU (rehearsal)
        if world <= torch.cuda.device_count():
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
            red_dev = torch.device("cpu")

    from encoder import inference as encoder
    from synthesizer.inference import Synthesizer
    from synthesizer.tacotron import set_dropout_stream, synth_tacotron_state_dict
    from wavernn_amd import inference as vocoder
    from wavernn_amd.base import hparams_for
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_state_dict

    rw = args.random_weights
    t0 = time.perf_counter()
    if rw is not None:
        encoder.load_model(None, device=dev, random_weights=rw)
        syn = Synthesizer(None, verbose=False, device=dev)
        from synthesizer.inference import build_tacotron
        sd = synth_tacotron_state_dict(build_tacotron("cpu"), rw + 1)
        sd["decoder.stop_proj.bias"] = torch.full_like(sd["decoder.stop_proj.bias"], -8.0)
        syn._state_dict = sd
        hp = hparams_for(args.vocoder_type)
        vocoder.load_model(None, verbose=False, device=local, model_type=args.vocoder_type,
                           state_dict=synth_state_dict(hp, args.vocoder_type, seed=rw + 2))
    else:
        encoder.load_model(args.enc_model_fpath, device=dev)
        syn = Synthesizer(args.syn_model_fpath, verbose=False, device=dev)
        vocoder.load_model(args.voc_model_fpath, device=local)
    syn.load()
    for _ in range(args.warmup):
        wv = encoder.preprocess_wav(synthetic_voice(seconds=1.0, seed=99), source_sr=16000)
        syn.synthesize_spectrograms(["warm up"], [encoder.embed_utterance(wv)], steps=20)
        mw = torch.zeros(sp.num_mels, 30, device=dev)  # >= 21 frames: the tail fade needs 20 hops
        hw = hparams_for(vocoder.get_model().model_type)
        vocoder.get_model().generate_batch([mw], True, hw.gen_target, hw.gen_overlap, hw.mu_law,
                                           sp.preemphasize)
    t_load = time.perf_counter() - t0

    mine = [i for i in range(args.utterances) if i % world == rank]
    texts = [TEXTS[i % len(TEXTS)] for i in mine]

    def run_pass():
        if args.seed is not None:
            torch.manual_seed(args.seed)
            vocoder.set_seed(args.seed)
            set_dropout_stream(args.seed)  # reproducible prenet dropout
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        # 1. speaker embedding of the reference utterance
        if args.ref_wav:
            ref = encoder.preprocess_wav(args.ref_wav)
        else:
            ref = encoder.preprocess_wav(synthetic_voice(seed=args.seed or 0), source_sr=16000)
        embed = encoder.embed_utterance(ref)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        # 2. spectrograms for this rank's texts (one Tacotron batch)
        specs = syn.synthesize_spectrograms(texts, [embed] * len(texts), steps=args.max_frames) if texts else []
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        # 3. vocoder: all of this rank's mels as one batch of fold rows (infer_waveform semantics)
        # utterance i draws noise stream (base + i) on whichever rank runs it, so the vocoder
        # output does not depend on the number of GPUs
        wavs = []
        model = vocoder.get_model()
        base = model.get_stream()
        if specs:
            hpv = hparams_for(model.model_type)
            mels = [torch.from_numpy(np.ascontiguousarray(s / sp.max_abs_value, dtype=np.float32)).to(dev)
                    for s in specs]
            wavs = model.generate_batch(mels, True, hpv.gen_target, hpv.gen_overlap, hpv.mu_law,
                                        sp.preemphasize, streams=[base + i for i in mine])
            if args.dump and rank == 0:
                rows = model.last_batch_rows
                nb = model.fold_shape(int(mels[0].shape[1]), True, hpv.gen_target, hpv.gen_overlap)[0]
                np.savez(args.dump, mel=mels[0].cpu().numpy(), rows=rows[:nb], wav=wavs[0],
                         seed=np.int64(args.seed if args.seed is not None else -1),
                         stream=np.int64(base + mine[0]), utterance=np.int64(mine[0]),
                         model_type=np.array(model.model_type),
                         weights_seed=np.int64(rw + 2 if rw is not None else -1))
        model.set_stream(base + args.utterances)
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        # 4. post: pad 1 s (demo_cli.py:197), trim / normalise like the reference
        outs = [encoder.preprocess_wav(np.pad(w, (0, sp.sample_rate), mode="constant").astype(np.float32))
                for w in wavs]
        t4 = time.perf_counter()
        return np.array([t1 - t0, t2 - t1, t3 - t2, t4 - t3, t4 - t0]), specs, wavs, outs

    # The same pass twice by default: the first pays the libraries' first use of every new
    # shape (MIOpen kernels of the encoder / Tacotron convolutions and GRUs; no cache persists
    # on a fresh box), the last is the steady state reported.
    totals = []
    for _ in range(max(1, args.repeat)):
        st, specs, wavs, outs = run_pass()
        totals.append(st[4])
    if args.out_dir:
        from scipy.io import wavfile
        os.makedirs(args.out_dir, exist_ok=True)
        for i, w in zip(mine, outs):
            wavfile.write(os.path.join(args.out_dir, "demo_output_%02d.wav" % i), sp.sample_rate,
                          w.astype(np.float32))
    stages = np.concatenate([st, [float(sum(len(w) for w in wavs))], [totals[0]]])
    if world > 1:
        ts = torch.tensor(stages[[0, 1, 2, 3, 4, 6]], device=red_dev, dtype=torch.float64)
        dist.all_reduce(ts, op=dist.ReduceOp.MAX)
        n = torch.tensor([stages[5]], device=red_dev, dtype=torch.float64)
        dist.all_reduce(n, op=dist.ReduceOp.SUM)
        t_ = ts.cpu().numpy()
        stages = np.concatenate([t_[:5], n.cpu().numpy(), t_[5:]])
    if rank == 0:
        audio_s = stages[5] / sp.sample_rate
        print(json.dumps({
            "demo": "encoder + tacotron + mi355x wavernn", "gpus": world,
            "utterances": args.utterances, "weights": "random(seed=%s)" % rw if rw is not None else "checkpoints",
            "vocoder": vocoder.get_model().model_type, "vocoder_engine": vocoder.get_model().last_engine(),
            "mel_frames": [int(s.shape[1]) for s in specs], "audio_seconds": round(audio_s, 3),
            "warmup_passes": args.warmup, "passes": max(1, args.repeat),
            "first_pass_total_seconds": round(stages[6], 4),
            "seconds": {"load": round(t_load, 3), "encoder": round(stages[0], 4),
                        "synthesizer": round(stages[1], 4), "vocoder": round(stages[2], 4),
                        "post": round(stages[3], 4), "total": round(stages[4], 4)},
            "xrtf_total": round(audio_s / stages[4], 2), "xrtf_vocoder": round(audio_s / stages[2], 2),
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
