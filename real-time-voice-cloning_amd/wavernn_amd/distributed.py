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

``split='folds'`` shards fold ROWS instead (``shard_folds``): the utterance-major list of all
fold rows is cut into ``world`` contiguous, equal pieces, so one utterance can span ranks -- the
single-utterance split of SURVEY §8e (fold groups per GPU, then the one gather). A rank runs
its pieces with ``wrnn_set_fold_ranges``; every row computes what it computes in a whole-
utterance call (conditioning positions and noise are keyed by the global fold index), so the
gathered rows, and the waveforms, equal the single-GPU ones bit for bit. Its use is latency:
a 1000-frame utterance's 18 rows on 2 GPUs run at 9 rows per GPU, on 3 or more at <= 6, where
every XCD group carries one row.
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


def shard_folds(n_frames, world, target, overlap, hop=200):
    """Fold-row sharding: rank r gets global rows [r R / world, (r + 1) R / world) of the
    utterance-major row list (R = all fold rows); returns per rank a list of (utt, lo, hi)
    segments, fold rows lo .. hi - 1 of utterance utt, in row order."""
    nf = [fold_rows(T, target, overlap, hop) for T in n_frames]
    R = sum(nf)
    cuts = [r * R // world for r in range(world + 1)]
    out = [[] for _ in range(world)]
    base = 0
    for u, n in enumerate(nf):
        for r in range(world):
            lo, hi = max(cuts[r], base), min(cuts[r + 1], base + n)
            if lo < hi:
                out[r].append((u, lo - base, hi - base))
        base += n
    return out


def infer_waveforms(mels, rows_fn, post_fn, target, overlap, seq_len, hop=200, device=None,
                    dst=0, threads=8, stream_base=0, dtype=None, out_rows=None, split='utterance'):
    """Vocode a list of mels across the ranks of the default process group.

    ``rows_fn(list_of_mels, streams) -> (rows, row_offsets)``: this rank's fold recurrence,
    ``rows`` a (n_rows, seq_len) int16 / float32 tensor on ``device``
    (``WaveRNN.generate_batch_device`` in production), ``row_offsets`` the first row of each
    utterance (+ the end). ``streams[j]`` is the noise stream of the j-th mel handed over:
    ``stream_base + i`` for utterance i of the GLOBAL list, whatever rank runs it -- so the
    output does not depend on the world size (the reference's CPU backend seeds every worker
    explicitly, vocoder/libwavernn/inference.py:106-108, :200-204). Callers advance their own
    stream counter by ``len(mels)`` afterwards, on every rank.
    ``split``: 'utterance' (whole utterances per rank, the default) or 'folds' (``shard_folds``;
    ``rows_fn`` then takes a third argument, the [(lo, hi)] fold range of each mel it is handed,
    and returns the rows of those ranges in order).
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
    if split not in ('utterance', 'folds'):
        raise ValueError(f"split must be 'utterance' or 'folds', not {split!r}")
    frames = [int(m.shape[-1]) for m in mels]
    if split == 'folds':
        return _infer_fold_split(mels, frames, rows_fn, post_fn, target, overlap, seq_len, hop,
                                 device, dst, threads, stream_base, dtype, out_rows, world, rank)
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


def _infer_fold_split(mels, frames, rows_fn, post_fn, target, overlap, seq_len, hop, device, dst,
                      threads, stream_base, dtype, out_rows, world, rank):
    import torch
    import torch.distributed as dist
    plan = shard_folds(frames, world, target, overlap, hop)
    nf = [fold_rows(T, target, overlap, hop) for T in frames]
    mine = plan[rank]
    if mine:
        rows, _ = rows_fn([mels[u] for u, _, _ in mine], [stream_base + u for u, _, _ in mine],
                          [(lo, hi) for _, lo, hi in mine])
        if rows.dtype != dtype:
            raise TypeError(f'rows_fn returned {rows.dtype}, expected {dtype}')
        if rows.shape[0] != sum(hi - lo for _, lo, hi in mine):
            raise ValueError(f'rows_fn returned {rows.shape[0]} rows for fold ranges {mine}')
    else:
        rows = None
    if world == 1:
        parts = [rows.cpu().numpy()]
    else:
        width = max(sum(hi - lo for _, lo, hi in p) for p in plan)
        dev = device if device is not None else (rows.device if rows is not None else torch.device('cpu'))
        if dist.get_backend() == 'gloo':
            dev = torch.device('cpu')
        buf = torch.zeros((width, seq_len), dtype=dtype, device=dev)
        if rows is not None:
            buf[:rows.shape[0]] = rows
        wire = buf.view(torch.uint8)
        bufs = [torch.empty_like(wire) for _ in range(world)] if rank == dst else None
        dist.gather(wire, bufs, dst=dst)
        if rank != dst:
            return None
        parts = [b.view(dtype).cpu().numpy() for b in bufs]
    full = [np.empty((n, seq_len), dtype=parts[0].dtype) for n in nf]
    for r in range(world):
        at = 0
        for u, lo, hi in plan[r]:
            full[u][lo:hi] = parts[r][at:at + hi - lo]
            at += hi - lo
    if out_rows is not None:
        for u in range(len(mels)):
            out_rows[u] = full[u]
    return _map(lambda u: post_fn(full[u], frames[u]), range(len(mels)), threads)


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
