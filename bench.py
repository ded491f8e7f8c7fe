"""Benchmark of the MI355X WaveRNN vocoder (BASELINE.json metric).

metric : WaveRNN audio samples/sec (xRTF @16kHz) -- output samples (T-1)*200 per utterance.
step   : one generate() over the per-GPU batch: upsample + conditioning + the full
         autoregressive fold recurrence on the GPU (mels already resident in HBM), labels
         copied to the host and the reference's f64 post-processing (cross-fade, mu-law,
         de-emphasis, fade-out) applied -- i.e. the whole job of vocoder.infer_waveform.
N=1    : BASELINE configs[1]: one 1000-frame mel, fatchord 9-bit mu-law RAW, target=11000,
         overlap=550 (18 folds x 12,100 steps).
N>1    : one process per GPU (torchrun); utterances are independent, so each rank runs its own
         shard (weak scaling, no collective on the data path); the fold rows are gathered to
         rank 0 (one RCCL gather) which post-processes every utterance (wavernn_amd.distributed).
         --utts-per-gpu 8 --gpus 8 is configs[3] (64 utterances on 8 GPUs).
         --split folds: strong scaling instead -- the --utts-per-gpu utterances of ONE job have
         their fold rows cut evenly over the N GPUs (single-utterance split, SURVEY §8e;
         wrnn_set_fold_ranges), the rows gathered to rank 0 as above; a latency mode.
Also reported: roofline of the dominant recurrent kernel (HIP events on its stream over the
timed region; HBM, fp32 and latency-floor fractions), the CPU baseline (oracle restatement of
the reference generate() on this host: the whole utterance on the default thread count, plus
bounded 1-thread and all-core legs; rank 0 after the timed region -- at N>1 on an utterance of the
last rank) and `parity`: the timed call's labels and waveform against that same oracle run (same
seed and noise stream). `config.lib_build` names the timed HIP library (SHA-256 prefix);
`roofline.traffic_lib_build` the library the PMC counters were read from.
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
    ap.add_argument('--prune', type=float, default=0.0,
                    help='prune the synthetic weights as the reference Pruner does at this '
                         'sparsity in 1x4 groups (vocoder/pruner.py; 0.9 = its target): the '
                         'block-sparse kernels run them (DESIGN.md §3.0g)')
    ap.add_argument('--sparse', default='auto', choices=['auto', '0', '1'],
                    help='block-sparse k_persist instances for pruned weights: by the planner '
                         '(auto), never (0), always (1) -- env WRNN_SPARSE')
    ap.add_argument('--split', default='utterance', choices=['utterance', 'folds'],
                    help="N>1 sharding: whole utterances per rank (weak scaling, default) or the "
                         "fold rows of the job's --utts-per-gpu utterances cut over the ranks "
                         "(strong scaling: one utterance's latency on N GPUs)")
    ap.add_argument('--engine', default='auto', choices=['auto', 'chain', 'persist'],
                    help='recurrence engine (include/wavernn_mi355x.h WRNN_ENGINE_*)')
    return ap.parse_args()


def workload_of(utts, frames, model, wname, target, overlap, prune=0.0):
    """The line's config.workload string; also the key under which tools/pmc_traffic.py files
    the counters of a workload (with the kernel name)."""
    return (f'{utts}x{frames}-frame mel per GPU, {model} {wname}, '
            f'batched folds target={target} overlap={overlap}' +
            (f', weights pruned {prune:.2f} in 1x4 blocks' if prune else ''))


def _pmc_traffic(kernel, workload):
    # WRNN_PMC_TRAFFIC: a table folded on the box from this build's own counter passes
    # (tools/measure_r04.sh), so the line's counters come from the binary it times
    path = os.environ.get('WRNN_PMC_TRAFFIC') or os.path.join(REPO, 'profiles', 'pmc_traffic.json')
    try:
        with open(path) as f:
            return json.load(f).get(f'{kernel}|{workload}')
    except (OSError, ValueError):
        return None


def lib_build_id():
    """First 16 hex digits of the SHA-256 of the loaded HIP library: names the binary a bench
    line (and a PMC pass, tools/pmc_traffic.py) measured."""
    import hashlib
    from wavernn_amd import _abi
    try:
        with open(_abi.LIB_PATH, 'rb') as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
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


# Latency model of the persistent recurrence: per step, `hops` in-group
# exchanges at the guide's one-to-one hand-off latency (MI355X_MICROARCH.md price list,
# handoff-1to1: 0.8 us idle for an 8-byte granule) plus the critical-path products of one
# workgroup at the fp32 vector peak (64 FLOP/clk/SIMD x 4 SIMDs x 2.4 GHz).
HANDOFF_US = 0.8
# the same hand-off with the endpoint CUs busy (the guide's row: 2 streaming waves -> 1.2 us for
# an 8-byte granule): the loaded floor, so the headroom claim is bounded from both sides
HANDOFF_LOADED_US = 1.2
CU_FP32_FLOP_PER_US = 64 * 4 * 2400.0
PERSIST_HOPS = {'fatchord-wavernn': 4, 'runtimeracer-wavernn': 8, 'geneing-wavernn': 2}


# MACs per row-step of the recurrent weight matrices
def latency_floor_us(model_type, hp, rows_per_group, n_classes, wide=False, handoff_us=HANDOFF_US):
    """Lower bound of one persistent step: exchange hops + critical products of one slot.
    Wide launches (kernels_persist_wide.hip) have one more hop (GRU1 is distributed) and run
    the products on 16-column MFMA tiles: 16 rows of work whatever the row count."""
    H, F = hp.rnn_dims, hp.fc_dims
    slots = 32
    if wide:
        rows_per_group = 16
    if model_type == 'fatchord-wavernn':      # GRU2 (3H x H) -> fc1 -> fc2 -> fc3
        crit = 3 * H * H + F * H + F * F + n_classes * F
    elif model_type == 'runtimeracer-wavernn':  # GRU2, GRU3, GRU4, fc1..fc5
        crit = 3 * (3 * H * H) + F * H + F * F + F * F + F * F + n_classes * F
    else:                                       # geneing: fc1 -> fc3
        crit = F * H + n_classes * F
    flop = 2.0 * crit * rows_per_group / slots
    hops = PERSIST_HOPS[model_type] + (1 if wide else 0)
    return hops * handoff_us + flop / CU_FP32_FLOP_PER_US, hops


def _oracle_run(args, sd, hp, mel, threads, max_steps=None, seed=0, stream=0, **kw):
    import torch
    from oracle.wavernn_oracle import OracleWaveRNN
    torch.set_num_threads(threads)
    o = OracleWaveRNN(sd, hp, args.model)
    m = torch.from_numpy(mel[None] / 4.0)
    t0 = time.perf_counter()
    r = o.generate(m, True, args.target, args.overlap, hp.mu_law, True, max_steps=max_steps,
                   seed=seed, stream=stream, **kw)
    r['t_wall'] = time.perf_counter() - t0
    return r


def _bounded_leg(args, sd, hp, mel, threads, seconds):
    """Oracle on `threads` host threads: upsample + the first k steps (k sized to ~seconds),
    the loop time extrapolated to all S steps."""
    probe = _oracle_run(args, sd, hp, mel, threads, max_steps=5)
    per_step = probe['t_loop'] / 5
    k = int(max(5, min(probe['S'], seconds / max(per_step, 1e-6))))
    r = _oracle_run(args, sd, hp, mel, threads, max_steps=k)
    t_total = r['t_prepare'] + r['t_loop'] * r['S'] / r['steps']
    samples = (args.frames - 1) * 200
    return dict(value=samples / t_total, unit='samples/s', cores=threads,
                sample=f"upsample + first {r['steps']} of {r['S']} steps ({r['B']} folds), loop "
                       f"extrapolated to all steps; {r['t_prepare'] + r['t_loop']:.1f}s measured")


def _cpu_share():
    """CPUs this process may actually use: the cgroup v2 quota (cpu.max) when one is set,
    else the affinity mask. (The GPU box shows every CPU of the machine in the mask but grants
    a share of them.)"""
    n_aff = len(os.sched_getaffinity(0))
    try:
        quota, period = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if quota != 'max':
            return max(1, min(n_aff, int(round(int(quota) / int(period))))), 'cgroup cpu.max'
    except (OSError, ValueError):
        pass
    return n_aff, 'affinity mask'


def _parity(r, gpu_rows, gpu_wav, seed, stream):
    """GPU fold rows / waveform of one utterance against the oracle run `r` (same seed, stream)."""
    import numpy as np
    parity = {'rows': int(r['B']), 'steps': int(r['S']), 'seed': seed, 'stream': stream}
    if r['labels'] is not None:
        diff = np.argwhere(gpu_rows != r['labels'])
        parity['labels_equal'] = bool(len(diff) == 0)
        parity['label_agreement'] = float((gpu_rows == r['labels']).mean())
        parity['first_divergence'] = (None if len(diff) == 0 else
                                      [int(v) for v in diff[np.argmin(diff[:, 1])]])
        parity['wave_bit_exact'] = bool(np.array_equal(gpu_wav, r['wav']))
    else:
        parity['samples_rms'] = float(np.sqrt(np.mean((gpu_rows.astype(np.float64) -
                                                        r['samples']) ** 2)))
        parity['wave_rms'] = float(np.sqrt(np.mean((gpu_wav - r['wav']) ** 2)))
        parity['tolerance'] = 1e-4
    return parity


def logit_gate(args, sd, hp, model, mel_dev, mel, gpu_rows, seed, stream):
    """Teacher-forced logit gate on the timed configuration (SURVEY §7 hard parts iii): the
    same call re-run with the kernels recording their pre-sampling logits at 6 steps (same seed
    and stream, so also a determinism check of the timed call's labels), against the oracle's
    logits at those steps; and the oracle's smallest top-1 / top-2 decision gap over EVERY
    (step, row) draw of the call -- how close the closest draw came to flipping."""
    import numpy as np
    import torch
    S = gpu_rows.shape[1]
    steps = sorted({0, 1, S // 4, S // 2, 3 * S // 4, S - 1})
    model.set_debug_steps(steps)
    try:
        rows, roff, _ = model.generate_batch_device([mel_dev], True, args.target, args.overlap,
                                                    streams=[stream])
        rerun = rows.cpu().numpy()[roff[0]:roff[1]]
        got = np.stack([model.debug_logits(t, range(rerun.shape[0])) for t in steps])
    finally:
        model.set_debug_steps([])
    r = _oracle_run(args, sd, hp, mel, torch.get_num_threads(), seed=seed, stream=stream,
                    record_logits=set(steps), track_margin=model.categorical, post=False)
    ref = np.stack([r['logits'][t] for t in steps])
    err = float(np.abs(got.astype(np.float64) - ref).max())
    out = {'steps': steps, 'max_abs_logit_err': err,
           'max_abs_logit': float(np.abs(ref).max()), 'tolerance': 1e-5,
           'rerun_identical': bool(np.array_equal(rerun, gpu_rows))}
    if 'margin' in r:
        out['min_top2_gap'] = r['margin']['min_gap']
        # how many times the logit error fits into the closest decision of the call
        out['gap_over_err'] = r['margin']['min_gap'] / err if err > 0 else None
        out['min_top2_gap_at'] = [r['margin']['step'], r['margin']['row']]
        out['min_top2_gap_over'] = f"{r['B']} rows x {r['S']} steps (log(p/q) top-1 - top-2)"
    return out


def parity_check(args, sd, hp, mel, gpu_rows, gpu_wav, seed, stream):
    """The oracle on the host (default threads) for one utterance: parity only, not timed."""
    import torch
    r = _oracle_run(args, sd, hp, mel, torch.get_num_threads(), seed=seed, stream=stream)
    return _parity(r, gpu_rows, gpu_wav, seed, stream)


def cpu_baseline(args, sd, hp, mel, gpu_rows, gpu_wav, seed, stream):
    """The oracle (torch-CPU restatement of the reference generate(), pinned bit-exact to the
    reference by tests/test_oracle_golden.py) on this host's cores.

    Leg 1 (`value`): the WHOLE workload of utterance 0 (all S steps, upsample, post) with
    torch's default thread count (OMP_NUM_THREADS: the box's CPU share), on the GPU run's own
    (seed, stream), so its labels / waveform are also the parity check of the timed GPU call.
    Legs 2 / 3: bounded samples with 1 thread and with every core in the affinity mask
    (all host cores and one core)."""
    import numpy as np
    import torch
    threads = torch.get_num_threads()
    n_aff = len(os.sched_getaffinity(0))
    r = _oracle_run(args, sd, hp, mel, threads, seed=seed, stream=stream)
    samples = (args.frames - 1) * 200
    parity = _parity(r, gpu_rows, gpu_wav, seed, stream)
    legs = [dict(value=samples / r['t_wall'], unit='samples/s', cores=threads,
                 sample=f"whole utterance: {r['B']} folds x {r['S']} steps + upsample + post, "
                        f"{r['t_wall']:.1f}s")]
    legs.append(_bounded_leg(args, sd, hp, mel, 1, args.cpu_seconds / 2))
    share, share_src = _cpu_share()
    if share > 1 and share != threads:
        legs.append(_bounded_leg(args, sd, hp, mel, share, args.cpu_seconds / 3))
    # (every CPU of the affinity mask when it exceeds the granted share is not timed: it only
    # oversubscribes the share -- 256 threads on 16 CPUs ran at 12 samples/s in round 2)
    torch.set_num_threads(threads)
    out = dict(legs[0], kind='port', cpu_model=_cpu_model(), affinity_cpus=n_aff,
               cpu_share=share, cpu_share_source=share_src, legs=legs)
    out['sample'] = (f"oracle.wavernn_oracle (torch-CPU restatement of reference generate()), "
                     f"{args.model} {args.mode} {args.bits}-bit, T={args.frames}, " + legs[0]['sample'])
    return out, parity


def main():
    args = parse()
    if args.sparse != 'auto':
        os.environ['WRNN_SPARSE'] = args.sparse
    import numpy as np
    import torch
    import torch.distributed as dist
    from wavernn_amd.model import WaveRNN
    from wavernn_amd.base import hparams_for
    from wavernn_amd.distributed import infer_waveforms, shard, shard_folds
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_state_dict, synth_mel

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # WRNN_BENCH_REHEARSE=1: every rank on cuda:0 over gloo -- a functional rehearsal of the N>1
    # path on a one-GPU box (its timings mean nothing: the ranks share one GPU)
    rehearse = os.environ.get('WRNN_BENCH_REHEARSE') == '1'
    if rehearse:
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if rehearse:
            dist.init_process_group('gloo')
        else:
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = torch.device('cuda', local)

    hp = hparams_for(args.model).copy(bits=args.bits, mode=args.mode)  # geneing RAW = Beta
    sd = synth_state_dict(hp, args.model, seed=0)
    if args.prune:
        from wavernn_amd.prune import prune_state_dict
        sd = prune_state_dict(sd, args.model, z=args.prune, group=4)
    model = WaveRNN(hp.rnn_dims, hp.fc_dims, hp.bits, hp.pad, hp.upsample_factors, sp.num_mels,
                    hp.compute_dims, hp.res_out_dims, hp.res_blocks, sp.hop_size, sp.sample_rate,
                    mode=hp.mode, model_type=args.model, device=local)
    model.load_state_dict(sd)
    seed = 1234
    model.set_seed(seed)
    model.set_engine(args.engine)
    U = args.utts_per_gpu
    folds = args.split == 'folds'
    n_utts = U if folds else U * world  # (fold split: the job's utterances, cut over the ranks)
    # every rank knows every utterance's length; only its own shard is resident in its HBM
    mels_host = [synth_mel(args.frames, seed=i) for i in range(n_utts)]
    if folds:
        fplan = shard_folds([args.frames] * n_utts, world, args.target, args.overlap)
        plan = [sorted({u for u, _, _ in p}) for p in fplan]
    else:
        plan = shard([args.frames] * n_utts, world, args.target, args.overlap)
    mine = set(plan[rank])
    mels = [torch.from_numpy((m / sp.max_abs_value).astype(np.float32)).to(dev) if i in mine
            else m for i, m in enumerate(mels_host)]
    S = model.fold_shape(args.frames, True, args.target, args.overlap)[1]
    if not args.no_timing:
        model.enable_stage_timing(True)
    last = {}
    rows_dtype = torch.int16 if model.categorical else torch.float32

    def rows_fn(ms, streams, ranges=None):
        # streams: the global utterance index offset by the step's base (distributed.py), so
        # every utterance draws the same noise whatever the world size; ranges: this rank's
        # fold rows of each (split='folds')
        out, roff, _ = model.generate_batch_device(ms, True, args.target, args.overlap,
                                                   streams=streams, fold_ranges=ranges)
        return out, roff

    def post_fn(rows, n_frames):
        return model.postprocess_rows(rows, n_frames, True, args.target, args.overlap, hp.mu_law,
                                      sp.preemphasize)

    def step():
        # the whole job: fold recurrence per rank, labels gathered to rank 0 (RCCL), f64 post
        base = model.get_stream()
        rows = {}
        w = infer_waveforms(mels, rows_fn, post_fn, args.target, args.overlap, S, device=dev,
                            stream_base=base, dtype=rows_dtype, out_rows=rows, split=args.split)
        model.set_stream(base + n_utts)  # every rank, whatever its shard
        last['base'], last['rows'] = base, rows
        return w

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
    dt_rank = dt
    if world > 1:
        t = torch.tensor([dt], device='cpu' if rehearse else dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    samples_per_step = n_utts * (args.frames - 1) * sp.hop_size
    if rank == 0:
        assert wavs is not None and sum(len(w) for w in wavs) == samples_per_step
    total_samples = samples_per_step * args.steps
    value = total_samples / dt

    wname = ('MOL' if hp.mode == 'MOL' else 'RAW (Beta)' if args.model == 'geneing-wavernn' and hp.mode == 'RAW'
             else f'{args.mode} {args.bits}-bit' + (' mu-law' if hp.mu_law else ''))
    workload = workload_of(U, args.frames, args.model, wname, args.target, args.overlap, args.prune)
    spi = model.sparse_info()
    roof = None
    us_rank = None
    info = model.stage_info() if not args.no_timing else []
    rows_per_gpu = U * model.fold_shape(args.frames, True, args.target, args.overlap)[0]
    if folds:
        rows_per_gpu = max(sum(hi - lo for _, lo, hi in p) for p in fplan)
        workload = workload.replace(' per GPU,', f' per job, fold rows split over {world} GPU(s),')
    if info:
        # dominant kernel = largest avg duration x launches
        dom_i = max(range(len(info)), key=lambda i: (info[i][3] if info[i][3] == info[i][3] else 0) * info[i][4])
        name, by, fl, us, n = info[dom_i]
        us_rank = us
        if world > 1:  # the slowest rank's launch bounds the job: roofline on the max over ranks
            t = torch.tensor([us], device='cpu' if rehearse else dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            us = float(t.item())
        achieved = by / (us * 1e-6) / 1e9 if us > 0 else None
        sfx = {'runtimeracer-wavernn': '_rr', 'geneing-wavernn': '_gen'}.get(args.model, '')
        kernel = {'persist': 'k_persist' + sfx, 'persist_wide': 'k_persist_wide' + sfx}.get(name, f'k_stage<{name}>')
        if name == 'persist' and spi['last_call']:
            kernel = 'k_persist (sparse)'  # the SP instances (pruned weights)
        roof = {'bound': 'hbm', 'kernel': kernel, 'achieved': achieved,
                'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': (achieved / HBM_PEAK_GBS) if achieved else None, 'traffic': None,
                'avg_us': us, 'launches_timed': n, 'alg_bytes_per_launch': by,
                'flops_per_launch': fl,
                'avg_us_over': ('max over ranks (all-reduced); rank 0: %.1f us' % us_rank
                                if world > 1 else 'one rank'),
                'fp32_tflops': fl / (us * 1e-6) / 1e12 if us > 0 else None,
                'fp32_frac': fl / (us * 1e-6) / 1e12 / FP32_PEAK_TFLOPS if us > 0 else None,
                'stages_us': {r[0]: round(r[3], 3) for r in info}}
        if name in ('persist', 'persist_wide'):
            # one launch per row batch runs all S steps; a row rotation runs
            # the call's rows over K launches of S / K steps on average, the time-sliced wide plan
            # (§3.0f) over launches of fewer steps: us_per_step is per step of a launch, and
            # call_us_per_step the kind's whole time in the call per step of S
            rot = model.rot_info() if name == 'persist' else (0, 0, 0)
            steps_launch = model.persist_steps(dom_i)
            roof['us_per_step'] = us / steps_launch
            roof['call_us_per_step'] = us * n / S
            roof['steps_per_launch'] = steps_launch
            if rot[0]:
                roof['rotation'] = {'launches': rot[0], 'steps_per_launch_hi_rows': rot[1],
                                    'steps_per_launch_lo_rows': rot[2],
                                    'us_per_step_note': 'call time / S (the rows rotate through groups of '
                                                        'q + 1 and q rows, each group at its own step rate)'}
            roof['launches_per_generate'] = sum(r[4] for r in info)
            # MACs per row-step as the runtime counts them (weights of I, rnn*, fc*)
            macs = sum(int(np.prod(v.shape)) for k, v in sd.items()
                       if k.startswith(('I.', 'rnn', 'fc')) and 'weight' in k)
            rows_l = fl / (steps_launch * 2.0 * macs) if S else 0
            nr = -(-int(round(rows_l)) // 8)
            floor, hops = latency_floor_us(args.model, hp, nr, model.n_classes,
                                           wide=name == 'persist_wide')
            floor_l, _ = latency_floor_us(args.model, hp, nr, model.n_classes, wide=name == 'persist_wide',
                                          handoff_us=HANDOFF_LOADED_US)
            roof['latency_floor_us'] = floor
            roof['latency_frac'] = floor / roof['us_per_step']
            roof['latency_floor_loaded_us'] = floor_l
            roof['latency_frac_loaded'] = floor_l / roof['us_per_step']
            roof['latency_model'] = (f'{hops} in-group hops x {HANDOFF_US} us (handoff-1to1, idle) or '
                                     f'x {HANDOFF_LOADED_US} us (loaded: endpoint CUs streaming) + '
                                     f'critical products of one slot at the fp32 vector peak, '
                                     f'{nr} rows per XCD group')
        # HBM traffic of the same kernel on the same workload from the committed PMC passes
        # (rocprofv3 cannot run inside this process; profiles/pmc_traffic.json names its source)
        pmc = _pmc_traffic(kernel, workload)
        if pmc:
            roof['traffic'] = pmc['traffic_bytes']
            roof['traffic_source'] = pmc['source']
            roof['traffic_lib_build'] = pmc.get('lib_build')
            roof['traffic_from_benched_build'] = pmc.get('lib_build') == lib_build_id()
            roof['traffic_note'] = pmc['correction']
            # counter-backed utilisation of the same kernel (SQ pass, tools/pmc_traffic.py):
            # MFMA pipe busy fraction over all 1024 SIMDs, LDS bank-conflict share, wave states
            for k in ('mfma_busy_frac', 'lds_conflict_frac', 'wait_frac', 'issue_stall_frac',
                      'active_frac', 'sq_source'):
                if k in pmc:
                    roof[k] = pmc[k]
    ranks = None
    if world > 1:
        # every rank's identity and timing (all-gathered), so an N > 1 line proves N distinct
        # GPUs and shows the slowest rank: world size as the process group sees it, hostname,
        # PCI address and UUID of the rank's device, its dominant kernel's average launch time
        # and its own wall time of the timed region
        import socket
        pr = torch.cuda.get_device_properties(dev)
        me = {'rank': rank, 'local_rank': local, 'hostname': socket.gethostname(),
              'pci': f'{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}',
              'uuid': str(getattr(pr, 'uuid', '')), 'kernel_avg_us': us_rank, 'wall_s': dt_rank}
        per = [None] * world
        dist.all_gather_object(per, me)
        timed = [r for r in per if r['kernel_avg_us'] is not None]
        ranks = {'world_size_pg': dist.get_world_size(), 'per_rank': per,
                 'distinct_devices': len({(r['hostname'], r['pci'], r['uuid']) for r in per}),
                 'slowest_rank_kernel': (max(timed, key=lambda r: r['kernel_avg_us'])['rank']
                                         if timed else None),
                 'slowest_rank_wall': max(per, key=lambda r: r['wall_s'])['rank']}
    fb = model.fallback_info()
    result = {
        'metric': 'WaveRNN audio samples/sec (xRTF @16kHz) at 1/2/4/8 MI355X vs CPU ref',
        'value': value, 'unit': 'samples/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': dt / args.steps * 1e3,
        'higher_is_better': True, 'scaling': 'strong' if folds and world > 1 else 'weak',
        'vs_baseline': None, 'dtype': 'f32',
        'data': 'synthetic (seeded random-init weights of the reference architecture, '
                'uniform[-4,4] mels)',
        'xrtf': value / sp.sample_rate,
        'config': {'workload': workload,
                   'utts_per_gpu': U, 'frames': args.frames, 'split': args.split,
                   'fold_rows_per_gpu': rows_per_gpu,
                   'parallelism': (f'{"fold rows" if folds else "utterances"} sharded over {world} '
                                   f'GPU(s); fold rows gathered to rank 0 (RCCL gather), f64 '
                                   f'post-processing on rank 0' if world > 1 else 'one GPU'),
                   'engine': model.last_engine(), 'persist_fallbacks': fb[0],
                   'sparse': {'prune': args.prune, 'image': spi['available'], 'ran': spi['last_call'],
                              'live_block_fraction': spi['density'], 'lds_list_fill_f4': spi['fill_f4']},
                   'lib_build': lib_build_id(),
                   'planner_rates': model.rates().splitlines()[0].replace('# source: ', '')},
        'roofline': roof,
        'cpu_baseline': None,
    }
    if ranks is not None:
        result['ranks'] = ranks
    if fb[0]:
        result['config']['fallback_reason'] = fb[1]
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        # parity of the last timed call: utterance 0's fold rows and waveform against the oracle
        gpu_rows = last['rows'][0]
        stream = last['base']
        # PCIe-inclusive rate of the drop-in host-buffer API (WaveRNN.generate as
        # infer_waveform calls it: host mel in, f64 waveform out, the reference's progress
        # callback at i % 100 == 0 -- one persistent launch, progress read from host-mapped
        # memory). Reported, never `value` (whose inputs are resident in HBM).
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
                    'progress callback at i % 100 == 0 (reference cadence)'}
        result['cpu_baseline'], result['parity'] = cpu_baseline(args, sd, hp, mels_host[0],
                                                                gpu_rows, wavs[0], seed, stream)
        result['parity']['logits'] = logit_gate(args, sd, hp, model, mels[0], mels_host[0],
                                                gpu_rows, seed, stream)
    elif rank == 0 and world > 1 and args.cpu_seconds > 0:
        # N > 1: the same CPU legs as N = 1, after the timed region and its barrier, on one
        # utterance of the LAST rank's shard (gathered over RCCL): the whole-utterance oracle leg
        # is also that utterance's parity check on its global stream (world-size invariance:
        # the same labels as at N = 1)
        u = plan[world - 1][-1] if folds else plan[world - 1][0]
        stream = last['base'] + u
        result['cpu_baseline'], result['parity'] = cpu_baseline(
            args, sd, hp, mels_host[u], last['rows'][u], wavs[u], seed, stream)
        result['parity'].update(utterance=u, from_rank=world - 1)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
