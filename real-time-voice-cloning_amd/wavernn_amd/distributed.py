"""Multi-GPU vocoding: independent utterances sharded over ranks (one process per GPU).

The reference has no multi-device inference path; utterances are fully
independent, so the data path shards them with no collective: each rank runs the fold
recurrence of its shard on its own GPU as one batch of fold rows. The one exchange is the
result collection: every rank's fold-row outputs (int16 labels for RAW / BITS, float32 samples
for MOL -- 2 or 4 bytes per row-step, ~3.5 MB for 8 x 1000-frame utterances) are gathered to
rank ``dst`` with one ``gather`` (RCCL over xGMI with the "nccl" backend, gloo on CPU), and
``dst`` runs the reference's f64 post-processing (cross-fade, mu-law, de-emphasis, fade;
fatchord_version.py:238-255) for every utterance on a host thread pool. Only ``dst`` receives
waveforms; the other ranks get None.

``shard(lengths, world)`` balances by work: every utterance costs S = target + 2*overlap
sequential steps regardless of length, and its number of fold rows grows with length, so the
greedy longest-first assignment balances rows per rank.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np


def fold_rows(n_frames, target, overlap, hop=200):
    """num_folds of fold_with_overlap (fatchord_version.py:316-327) for an n_frames mel."""
    L = n_frames * hop
    nf = (L - overlap) // (target + overlap)
    if L - (nf * (overlap + target) + overlap) != 0:
        nf += 1
    return nf


def shard(n_frames, world, target, overlap, hop=200):
    """Assign utterance indices to ranks, longest (most fold rows) first; returns list per rank."""
    order = sorted(range(len(n_frames)), key=lambda i: (-fold_rows(n_frames[i], target, overlap, hop), i))
    load = [0] * world
    out = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        out[r].append(i)
        load[r] += fold_rows(n_frames[i], target, overlap, hop)
    for r in range(world):
        out[r].sort()
    return out


def infer_waveforms(mels, rows_fn, post_fn, target, overlap, seq_len, hop=200, device=None,
                    dst=0, threads=8, stream_base=0, dtype=None, out_rows=None):
    """Vocode a list of mels across the ranks of the default process group.

    ``rows_fn(list_of_mels, streams) -> (rows, row_offsets)``: this rank's fold recurrence,
    ``rows`` a (n_rows, seq_len) int16 / float32 tensor on ``device``
    (``WaveRNN.generate_batch_device`` in production), ``row_offsets`` the first row of each
    utterance (+ the end). ``streams[j]`` is the noise stream of the j-th mel handed over:
    ``stream_base + i`` for utterance i of the GLOBAL list, whatever rank runs it -- so the
    output does not depend on the world size (the reference's CPU backend seeds every worker
    explicitly, vocoder/libwavernn/inference.py:106-108, :200-204). Callers advance their own
    stream counter by ``len(mels)`` afterwards, on every rank.
    ``post_fn(rows_np, n_frames) -> f64 waveform``: the host post-processing of one utterance
    (``WaveRNN.postprocess_rows``). ``dtype``: the rows' torch dtype (int16 for categorical
    models, float32 for MOL / Beta) -- every rank must gather buffers of the same byte size,
    including a rank whose shard is empty; default int16. ``out_rows``: a dict that receives
    each utterance's gathered (num_folds, seq_len) host rows on ``dst``.
    Returns the waveforms in input order on ``dst`` (None on the other ranks; every waveform
    on a single process).
    """
    import torch
    import torch.distributed as dist
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    dtype = dtype if dtype is not None else torch.int16
    if not mels:  # every rank sees the same (empty) list: nothing to run or gather
        return [] if rank == dst or world == 1 else None
    frames = [int(m.shape[-1]) for m in mels]
    plan = shard(frames, world, target, overlap, hop)
    rows_of = [sum(fold_rows(frames[i], target, overlap, hop) for i in p) for p in plan]
    mine = plan[rank]
    if mine:
        rows, roff = rows_fn([mels[i] for i in mine], [stream_base + i for i in mine])
        if rows.dtype != dtype:
            raise TypeError(f'rows_fn returned {rows.dtype}, expected {dtype}')
    else:
        rows, roff = None, [0]
    if world == 1:
        host = rows.cpu().numpy()
        if out_rows is not None:
            for j, i in enumerate(mine):
                out_rows[i] = host[roff[j]:roff[j + 1]]
        return _map(lambda j: post_fn(host[roff[j]:roff[j + 1]], frames[mine[j]]),
                    range(len(mine)), threads)
    # one gather of equal-shaped buffers (rows padded to the largest shard) to dst
    width = max(rows_of)
    dev = device if device is not None else (rows.device if rows is not None else torch.device('cpu'))
    if dist.get_backend() == 'gloo':  # gloo gathers host tensors (CPU test, 1-GPU rehearsal)
        dev = torch.device('cpu')
    buf = torch.zeros((width, seq_len), dtype=dtype, device=dev)
    if rows is not None:
        buf[:rows.shape[0]] = rows
    # as bytes: RCCL / NCCL and gloo have no int16 type
    wire = buf.view(torch.uint8)
    bufs = [torch.empty_like(wire) for _ in range(world)] if rank == dst else None
    dist.gather(wire, bufs, dst=dst)
    if rank != dst:
        return None
    jobs = []
    for r in range(world):
        host = bufs[r].view(dtype).cpu().numpy()
        at = 0
        for i in plan[r]:
            nf = fold_rows(frames[i], target, overlap, hop)
            jobs.append((i, host[at:at + nf]))
            at += nf
    if out_rows is not None:
        for i, rws in jobs:
            out_rows[i] = rws
    out = [None] * len(mels)
    for i, w in zip([j[0] for j in jobs], _map(lambda j: post_fn(j[1], frames[j[0]]), jobs, threads)):
        out[i] = w
    return out


_POOL = {}


def _map(fn, items, threads):
    """fn over items: inline for one item, else on a process-wide thread pool (created once:
    a pool per call costs about a millisecond of thread start-up on the bench's path)."""
    items = list(items)
    if len(items) <= 1 or threads <= 1:
        return [fn(x) for x in items]
    if threads not in _POOL:
        _POOL[threads] = ThreadPoolExecutor(threads)
    return list(_POOL[threads].map(fn, items))
