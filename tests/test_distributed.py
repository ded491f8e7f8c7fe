"""Multi-process path (CPU, gloo, world_size 2): utterance sharding + result collection.

The per-rank fold recurrence here is the oracle on tiny inputs (test infrastructure) and the
host post-processing is the product's (wavernn_amd.audio with the C-ABI library's host loops);
int16 labels are gathered to rank 0, which post-processes every utterance. On the GPU box
bench.py --gpus N drives the same infer_waveforms() with WaveRNN.generate_batch_device on the
nccl (RCCL) backend.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def test_shard_balances_rows_and_covers_all():
    from wavernn_amd.distributed import shard, fold_rows
    frames = [1000, 200, 1000, 50, 700, 1000, 30, 400]
    for world in (1, 2, 3, 8):
        plan = shard(frames, world, 11000, 550)
        flat = sorted(i for p in plan for i in p)
        assert flat == list(range(len(frames)))
        loads = [sum(fold_rows(frames[i], 11000, 550) for i in p) for p in plan]
        assert max(loads) - min(loads) <= max(fold_rows(f, 11000, 550) for f in frames)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _hp(mode):
    from wavernn_amd.hparams import wavernn_fatchord
    return wavernn_fatchord.copy(bits=9, mode=mode)


FRAMES = {'RAW': [22, 30, 25], 'MOL': [24, 21]}
STREAM_BASE = 7  # the callers' stream counter before the call (bench: model.get_stream())


def _worker(rank, world, port, q, mode, split='utterance'):
    import sys
    import torch
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), 'real-time-voice-cloning_amd'))
    sys.path.insert(0, os.path.dirname(here))
    torch.set_num_threads(1)
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from oracle.wavernn_oracle import oracle_infer_waveform
    from wavernn_amd import _abi
    from wavernn_amd.audio import postprocess
    from wavernn_amd.distributed import infer_waveforms
    from wavernn_amd.synth import synth_state_dict, synth_mel
    hp = _hp(mode)
    sd = synth_state_dict(hp, 'fatchord-wavernn', seed=1)
    mels = [synth_mel(T, seed=10 + i) for i, T in enumerate(FRAMES[mode])]
    lib = _abi.load_library()
    raw = mode == 'RAW'
    ran = []

    def rows_fn(ms, streams, ranges=None):
        # one stream per utterance of the GLOBAL list, as WaveRNN.generate_batch_device gets it;
        # fold split: the rows lo .. hi - 1 of each (the ABI's wrnn_set_fold_ranges contract,
        # pinned against whole calls on the GPU by test_gpu_fold_split.py)
        ran.extend(streams if ranges is None else list(zip(streams, ranges)))
        outs = [oracle_infer_waveform(sd, hp, 'fatchord-wavernn', m, target=400, overlap=50,
                                      seed=5, stream=s, post=False)['labels' if raw else 'samples']
                for m, s in zip(ms, streams)]
        if ranges is not None:
            outs = [o[lo:hi] for o, (lo, hi) in zip(outs, ranges)]
        roff = np.cumsum([0] + [o.shape[0] for o in outs]).tolist()
        return torch.from_numpy(np.concatenate(outs)), roff

    def post_fn(rows, n_frames):
        if raw:
            smp = (np.float32(2) * rows.astype(np.float32)) / np.float32(511.) - np.float32(1.)
            return postprocess(smp, True, 400, 50, True, True, 512, (n_frames - 1) * 200, 200,
                               labels=rows, lib=lib)
        return postprocess(rows, True, 400, 50, False, True, 30, (n_frames - 1) * 200, 200,
                           lib=lib)
    wavs = infer_waveforms(mels, rows_fn, post_fn, 400, 50, seq_len=500,
                           stream_base=STREAM_BASE, dtype=torch.int16 if raw else torch.float32,
                           split=split)
    q.put((rank, sorted(ran)))
    if rank == 0:
        q.put([w.tolist() for w in wavs])
    else:
        assert wavs is None
    dist.destroy_process_group()


def _run(world, mode, split='utterance'):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode, split)) for r in range(world)]
    for p in procs:
        p.start()
    streams, got = {}, None
    for _ in range(world + 1):
        item = q.get(timeout=300)
        if isinstance(item, tuple):
            streams[item[0]] = item[1]
        else:
            got = item
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return streams, got


def _single_process(mode):
    from oracle.wavernn_oracle import oracle_infer_waveform
    from wavernn_amd.synth import synth_state_dict, synth_mel
    hp = _hp(mode)
    sd = synth_state_dict(hp, 'fatchord-wavernn', seed=1)
    return [oracle_infer_waveform(sd, hp, 'fatchord-wavernn', synth_mel(T, seed=10 + i),
                                  target=400, overlap=50, seed=5, stream=STREAM_BASE + i)['wav']
            for i, T in enumerate(FRAMES[mode])]


def test_two_rank_gather_equals_single_process():
    """N = 2 == N = 1 bit for bit: utterance i draws stream base + i on whichever rank runs it
    (world-size invariant output), and every stream is used exactly once."""
    streams, got = _run(2, 'RAW')
    ref = _single_process('RAW')
    n = len(FRAMES['RAW'])
    assert sorted(s for r in streams.values() for s in r) == [STREAM_BASE + i for i in range(n)]
    for i in range(n):
        assert np.array_equal(np.asarray(got[i]), ref[i])


def test_three_ranks_two_mol_utterances_empty_shard():
    """More ranks than utterances: the empty rank still gathers a buffer of the MOL rows'
    dtype (float32), so the gather matches the others' byte size; output == one process."""
    streams, got = _run(3, 'MOL')
    assert [] in streams.values()
    ref = _single_process('MOL')
    for i in range(len(FRAMES['MOL'])):
        assert np.array_equal(np.asarray(got[i]), ref[i])


def test_empty_utterance_list():
    from wavernn_amd.distributed import infer_waveforms
    assert infer_waveforms([], None, None, 400, 50, seq_len=500) == []


def test_shard_folds_cuts_rows_evenly():
    from wavernn_amd.distributed import shard_folds, fold_rows
    frames = [1000, 200, 1000, 50, 700]
    nf = [fold_rows(f, 11000, 550) for f in frames]
    for world in (1, 2, 3, 4, 8, 64):
        plan = shard_folds(frames, world, 11000, 550)
        sizes = [sum(hi - lo for _, lo, hi in p) for p in plan]
        assert max(sizes) - min(sizes) <= 1 and sum(sizes) == sum(nf)
        # every fold row of every utterance exactly once, in utterance-major order
        flat = [(u, f) for p in plan for u, lo, hi in p for f in range(lo, hi)]
        assert flat == [(u, f) for u, n in enumerate(nf) for f in range(n)]
    # one 1000-frame utterance (C2: 18 rows) over 2 / 4 ranks
    assert shard_folds([1000], 2, 11000, 550) == [[(0, 0, 9)], [(0, 9, 18)]]
    assert [sum(hi - lo for _, lo, hi in p) for p in shard_folds([1000], 4, 11000, 550)] == [4, 5, 4, 5]


def test_two_rank_fold_split_equals_single_process():
    """split='folds': the 3 RAW utterances' fold rows cut evenly over 2 ranks (one utterance
    spans both), gathered and re-assembled on rank 0 -- waveforms == one process bit for bit,
    and each rank ran the ranges shard_folds assigned it."""
    from wavernn_amd.distributed import shard_folds
    streams, got = _run(2, 'RAW', split='folds')
    ref = _single_process('RAW')
    plan = shard_folds(FRAMES['RAW'], 2, 400, 50)
    for r in range(2):
        assert streams[r] == sorted((STREAM_BASE + u, (lo, hi)) for u, lo, hi in plan[r])
    assert any(u == plan[1][0][0] for u, _, _ in plan[0])  # an utterance spans the ranks
    for i in range(len(FRAMES['RAW'])):
        assert np.array_equal(np.asarray(got[i]), ref[i])


def test_fold_split_single_process_reassembles_float_rows():
    """split='folds' without a process group (world 1) on float32 (MOL-type) rows: rows_fn sees
    every utterance's whole range and post_fn gets each utterance's rows back in fold order."""
    import torch
    from wavernn_amd.distributed import infer_waveforms, fold_rows
    frames = [30, 22, 41]
    nf = [fold_rows(T, 400, 50) for T in frames]
    mels = [np.zeros((80, T), np.float32) for T in frames]
    seen = []

    def rows_fn(ms, streams, ranges):
        seen.append((streams, ranges))
        # row f of utterance u holds u * 100 + f in every step
        return torch.cat([torch.arange(lo, hi, dtype=torch.float32)[:, None].repeat(1, 500) + 100 * (s - 3)
                          for s, (lo, hi) in zip(streams, ranges)]), None

    got = infer_waveforms(mels, rows_fn, lambda rows, T: rows[:, 0].copy(), 400, 50, seq_len=500,
                          stream_base=3, dtype=torch.float32, split='folds')
    assert seen == [([3, 4, 5], [(0, n) for n in nf])]
    for u, n in enumerate(nf):
        assert np.array_equal(got[u], 100 * u + np.arange(n, dtype=np.float32))


def test_fold_split_rejects_unknown_mode():
    from wavernn_amd.distributed import infer_waveforms
    with pytest.raises(ValueError):
        infer_waveforms([np.zeros((80, 30), np.float32)], None, None, 400, 50, seq_len=500,
                        split='rows')
