"""Single-utterance latency of a fold split over K GPUs, measured on ONE MI355X.

A K-GPU fold split (wavernn_amd.distributed, split='folds') runs each rank's contiguous piece of
the utterance's fold rows (wrnn_set_fold_ranges) independently, then gathers the int16 rows to
rank 0 (one RCCL gather of <= 18 x 12,100 x 2 B = 436 KB) for the f64 post-processing. The
ranks share nothing until that gather, so the job's latency is the slowest piece's device time
plus the gather plus the post. This tool times, on one GPU, every rank's piece for K = 1..8
(the pieces of shard_folds), the whole call, and the host post of the full rows; the RCCL gather
is not timed here (no multi-GPU node; xGMI moves 436 KB in a few microseconds, the collective's
launch costs tens). Every piece's rows are checked bit for bit against the whole call's.

usage: python tools/split_latency.py [--frames 1000] [--reps 5] > out.jsonl
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'real-time-voice-cloning_amd'))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--frames', type=int, default=1000)
    ap.add_argument('--target', type=int, default=11000)
    ap.add_argument('--overlap', type=int, default=550)
    ap.add_argument('--bits', type=int, default=9)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--kmax', type=int, default=8)
    args = ap.parse_args()
    import numpy as np
    import torch
    from wavernn_amd.base import hparams_for
    from wavernn_amd.distributed import shard_folds
    from wavernn_amd.hparams import sp
    from wavernn_amd.model import WaveRNN
    from wavernn_amd.synth import synth_mel, synth_state_dict
    hp = hparams_for('fatchord-wavernn').copy(bits=args.bits, mode='RAW')
    m = WaveRNN(hp.rnn_dims, hp.fc_dims, hp.bits, hp.pad, hp.upsample_factors, sp.num_mels,
                hp.compute_dims, hp.res_out_dims, hp.res_blocks, sp.hop_size, sp.sample_rate,
                mode=hp.mode, model_type='fatchord-wavernn', device=0)
    m.load_state_dict(synth_state_dict(hp, 'fatchord-wavernn', seed=0))
    m.set_seed(1234)
    mel = [torch.from_numpy((synth_mel(args.frames, seed=0) / sp.max_abs_value).astype(np.float32)).cuda()]

    def run(rng):
        torch.cuda.synchronize()
        t = time.perf_counter()
        out, _, _ = m.generate_batch_device(mel, True, args.target, args.overlap, streams=[0],
                                            fold_ranges=None if rng is None else [rng])
        torch.cuda.synchronize()
        return out, time.perf_counter() - t

    run(None)
    full, _ = run(None)
    full = full.cpu().numpy()
    whole = min(run(None)[1] for _ in range(args.reps))
    tp = time.perf_counter()
    for _ in range(args.reps):
        m.postprocess_rows(full, args.frames, True, args.target, args.overlap, hp.mu_law, sp.preemphasize)
    post = (time.perf_counter() - tp) / args.reps
    nsamp = (args.frames - 1) * sp.hop_size
    print(json.dumps({'k': 1, 'whole_call_ms': whole * 1e3, 'post_ms': post * 1e3,
                      'latency_ms': (whole + post) * 1e3, 'samples': nsamp,
                      'xrtf': nsamp / sp.sample_rate / (whole + post)}), flush=True)
    for k in range(2, args.kmax + 1):
        pieces = [(lo, hi) for p in shard_folds([args.frames], k, args.target, args.overlap)
                  for _, lo, hi in p]
        times, plans, exact = [], [], True
        for rng in pieces:
            out, _ = run(rng)
            exact &= bool(np.array_equal(out.cpu().numpy(), full[rng[0]:rng[1]]))
            times.append(min(run(rng)[1] for _ in range(args.reps)))
            plans.append(m.plan_info())
        slow = max(times)
        print(json.dumps({'k': k, 'pieces': pieces, 'piece_ms': [t * 1e3 for t in times],
                          'slowest_piece_ms': slow * 1e3, 'post_ms': post * 1e3,
                          'latency_ms_excl_gather': (slow + post) * 1e3,
                          'xrtf_excl_gather': nsamp / sp.sample_rate / (slow + post),
                          'speedup_vs_1gpu': (whole + post) / (slow + post),
                          'rows_bit_exact_vs_whole': exact,
                          'plans': [[list(x) for x in p] for p in plans]}), flush=True)


if __name__ == '__main__':
    main()
