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


def _worker(rank, world, port, q):
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
    from wavernn_amd.hparams import wavernn_fatchord
    from wavernn_amd.synth import synth_state_dict, synth_mel
    hp = wavernn_fatchord.copy(bits=9)
    sd = synth_state_dict(hp, 'fatchord-wavernn', seed=1)
    mels = [synth_mel(T, seed=10 + i) for i, T in enumerate([22, 30, 25])]
    lib = _abi.load_library()

    def rows_fn(ms):
        outs = [oracle_infer_waveform(sd, hp, 'fatchord-wavernn', m, target=400, overlap=50,
                                      seed=5, stream=0, post=False)['labels'] for m in ms]
        roff = np.cumsum([0] + [o.shape[0] for o in outs]).tolist()
        return torch.from_numpy(np.concatenate(outs)), roff

    def post_fn(rows, n_frames):
        smp = (np.float32(2) * rows.astype(np.float32)) / np.float32(511.) - np.float32(1.)
        return postprocess(smp, True, 400, 50, True, True, 512, (n_frames - 1) * 200, 200,
                           labels=rows, lib=lib)
    wavs = infer_waveforms(mels, rows_fn, post_fn, 400, 50, seq_len=500)
    if rank == 0:
        q.put([w.tolist() for w in wavs])
    else:
        assert wavs is None
    dist.destroy_process_group()


def test_two_rank_gather_equals_single_process():
    from oracle.wavernn_oracle import oracle_infer_waveform
    from wavernn_amd.hparams import wavernn_fatchord
    from wavernn_amd.synth import synth_state_dict, synth_mel
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    hp = wavernn_fatchord.copy(bits=9)
    sd = synth_state_dict(hp, 'fatchord-wavernn', seed=1)
    for i, T in enumerate([22, 30, 25]):
        ref = oracle_infer_waveform(sd, hp, 'fatchord-wavernn', synth_mel(T, seed=10 + i),
                                    target=400, overlap=50, seed=5, stream=0)['wav']
        assert np.array_equal(np.asarray(got[i]), ref)
