"""Benchmark of the MI355X WaveRNN vocoder (BASELINE.json metric).

metric : WaveRNN audio samples/sec (xRTF @16kHz) -- output samples (T-1)*200 per utterance.
step   : one generate() over the per-GPU batch: upsample + conditioning + the full
         autoregressive fold recurrence on the GPU (mels already resident in HBM), labels
         copied to the host and the reference's f64 post-processing (cross-fade, mu-law,
         de-emphasis, fade-out) applied -- i.e. the whole job of vocoder.infer_waveform.
N=1    : BASELINE configs[1]: one 1000-frame mel, fatchord 9-bit mu-law RAW, target=11000,
         overlap=550 (18 folds x 12,100 steps).
N>1    : one process per GPU (torchrun); utterances are independent, so each rank runs its own
         (weak scaling, no data-path collective); --utts-per-gpu 8 --gpus 8 is configs[3]
         (64 utterances on 8 GPUs).
Also reported: roofline of the dominant recurrent kernel (in-kernel s_memrealtime stamps over
the timed region) and the CPU baseline (oracle restatement of the reference generate(), timed
on this host on a bounded sample of the same workload, rank 0, N=1 only).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'real-time-voice-cloning_amd'))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--utts-per-gpu', type=int, default=1)
    ap.add_argument('--frames', type=int, default=1000)
    ap.add_argument('--model', default='fatchord-wavernn')
    ap.add_argument('--mode', default='RAW')
    ap.add_argument('--bits', type=int, default=9)
    ap.add_argument('--target', type=int, default=11000)
    ap.add_argument('--overlap', type=int, default=550)
    ap.add_argument('--cpu-seconds', type=float, default=15.0,
                    help='CPU-baseline sample budget (0 disables)')
    ap.add_argument('--no-timing', action='store_true', help='disable kernel timing')
    ap.add_argument('--engine', default='auto', choices=['auto', 'chain', 'persist'],
                    help='recurrence engine (include/wavernn_mi355x.h WRNN_ENGINE_*)')
    return ap.parse_args()


def _pmc_traffic(kernel, workload):
    try:
        with open(os.path.join(REPO, 'profiles', 'pmc_traffic.json')) as f:
            return json.load(f).get(f'{kernel}|{workload}')
    except (OSError, ValueError):
        return None


def _cpu_model():
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def cpu_baseline(args, sd, hp, mel):
    """Oracle (torch-CPU restatement of the reference generate) on a bounded sample."""
    import torch
    from oracle.wavernn_oracle import OracleWaveRNN
    cores = torch.get_num_threads()
    o = OracleWaveRNN(sd, hp, args.model)
    m = torch.from_numpy(mel[None] / 4.0)
    # calibrate: time 50 steps, then size the sample to ~cpu_seconds
    probe = o.generate(m, True, args.target, args.overlap, hp.mu_law, True, max_steps=50)
    per_step = probe['t_loop'] / 50
    k = int(max(100, min(probe['S'], args.cpu_seconds / max(per_step, 1e-6))))
    r = o.generate(m, True, args.target, args.overlap, hp.mu_law, True, max_steps=k)
    S = r['S']
    t_total = r['t_prepare'] + r['t_loop'] * S / r['steps']
    samples = (args.frames - 1) * 200
    return dict(value=samples / t_total, unit='samples/s', cores=cores, kind='port',
                cpu_model=_cpu_model(), affinity_cpus=len(os.sched_getaffinity(0)),
                sample=f"oracle.wavernn_oracle (torch-CPU restatement of reference generate()), "
                       f"{args.model} {args.mode} {args.bits}-bit, T={args.frames}: upsample + first "
                       f"{r['steps']} of {S} steps ({r['B']} folds), loop time extrapolated to all "
                       f"steps; {r['t_prepare'] + r['t_loop']:.1f}s measured")


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist
    from wavernn_amd.model import WaveRNN
    from wavernn_amd.base import hparams_for
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_state_dict, synth_mel

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = torch.device('cuda', local)

    mode = 'BITS' if args.model == 'geneing-wavernn' and args.mode == 'RAW' else args.mode
    hp = hparams_for(args.model).copy(bits=args.bits, mode=mode)
    sd = synth_state_dict(hp, args.model, seed=0)
    model = WaveRNN(hp.rnn_dims, hp.fc_dims, hp.bits, hp.pad, hp.upsample_factors, sp.num_mels,
                    hp.compute_dims, hp.res_out_dims, hp.res_blocks, sp.hop_size, sp.sample_rate,
                    mode=hp.mode, model_type=args.model, device=local)
    model.load_state_dict(sd)
    model.set_seed(1234)
    model.set_engine(args.engine)
    U = args.utts_per_gpu
    mels_host = [synth_mel(args.frames, seed=rank * U + u) for u in range(U)]
    mels_dev = [torch.from_numpy(m / sp.max_abs_value).to(dev) for m in mels_host]
    if not args.no_timing:
        model.enable_stage_timing(True)

    def step():
        return model.generate_batch(mels_dev, True, args.target, args.overlap, hp.mu_law,
                                    sp.preemphasize)

    for _ in range(args.warmup):
        wavs = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        wavs = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    samples_per_step = sum(len(w) for w in wavs)
    total_samples = samples_per_step * args.steps * world
    value = total_samples / dt

    workload = (f'{U}x{args.frames}-frame mel per GPU, {args.model} {args.mode} {args.bits}-bit mu-law, '
                f'batched folds target={args.target} overlap={args.overlap}')
    roof = None
    info = model.stage_info() if not args.no_timing else []
    if info:
        # dominant kernel = largest avg duration x launches
        dom = max(info, key=lambda r: (r[3] if r[3] == r[3] else 0) * r[4])
        name, by, fl, us, n = dom
        achieved = by / (us * 1e-6) / 1e9 if us > 0 else None
        kernel = 'k_persist' if name == 'persist' else f'k_stage<{name}>'
        roof = {'bound': 'hbm', 'kernel': kernel, 'achieved': achieved,
                'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': (achieved / HBM_PEAK_GBS) if achieved else None, 'traffic': None,
                'avg_us': us, 'launches_timed': n, 'alg_bytes_per_launch': by,
                'flops_per_launch': fl,
                'fp32_tflops': fl / (us * 1e-6) / 1e12 if us > 0 else None,
                'stages_us': {r[0]: round(r[3], 3) for r in info}}
        if name == 'persist':  # no progress callback -> one launch per row batch runs all S steps
            S = model.fold_shape(args.frames, True, args.target, args.overlap)[1]
            roof['us_per_step'] = us / S
            roof['launches_per_generate'] = n  # stage timing keeps the last generate's launches
        # HBM traffic of the same kernel on the same workload from the committed PMC passes
        # (rocprofv3 cannot run inside this process; profiles/pmc_traffic.json names its source)
        pmc = _pmc_traffic(kernel, workload)
        if pmc:
            roof['traffic'] = pmc['traffic_bytes']
            roof['traffic_source'] = pmc['source']
            roof['traffic_note'] = pmc['correction']
    result = {
        'metric': 'WaveRNN audio samples/sec (xRTF @16kHz) at 1/2/4/8 MI355X vs CPU ref',
        'value': value, 'unit': 'samples/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': dt / args.steps * 1e3,
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f32',
        'data': 'synthetic (seeded random-init weights of the reference architecture, '
                'uniform[-4,4] mels)',
        'xrtf': value / sp.sample_rate,
        'config': {'workload': workload,
                   'utts_per_gpu': U, 'frames': args.frames,
                   'fold_rows_per_gpu': U * model.fold_shape(args.frames, True, args.target,
                                                             args.overlap)[0],
                   'parallelism': f'utterances sharded over {world} GPU(s), no collective',
                   'engine': model.last_engine()},
        'roofline': roof,
        'cpu_baseline': None,
    }
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        # PCIe-inclusive rate of the drop-in host-buffer API (WaveRNN.generate as
        # infer_waveform calls it: host mel in, f64 waveform out, progress callback every 100
        # steps, so the persistent engine runs in launches of 1000 steps). Reported, never
        # `value` (whose inputs are resident in HBM).
        mel0 = (mels_host[0] / sp.max_abs_value).astype(np.float32)
        model.generate(mel0, True, args.target, args.overlap, hp.mu_law, sp.preemphasize,
                       progress_callback=lambda *a: None)
        th = time.perf_counter()
        wav = model.generate(mel0, True, args.target, args.overlap, hp.mu_law,
                             sp.preemphasize, progress_callback=lambda *a: None)
        th = time.perf_counter() - th
        result['dropin_host_io'] = {
            'value': len(wav) / th, 'unit': 'samples/s', 'ms': th * 1e3,
            'path': 'WaveRNN.generate(host mel) -> f64 waveform: H2D mel, labels D2H, '
                    'progress callback every 100 steps (persist launches of 1000 steps)'}
        result['cpu_baseline'] = cpu_baseline(args, sd, hp, mels_host[0])
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
