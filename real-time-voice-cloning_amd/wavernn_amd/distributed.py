"""Multi-GPU vocoding: independent utterances sharded over ranks (one process per GPU).

The reference has no multi-device inference path; utterances are fully
independent, so the MI355X build shards them with no data-path collective: each rank vocodes
its shard on its own GPU as one batch of fold rows, and the only exchange is collecting the
finished waveforms on rank 0 (one all-gather of fixed, known sizes -- RCCL over xGMI with the
"nccl" backend, or gloo on CPU).

``shard(lengths, world)`` balances by work: every utterance costs S = target + 2*overlap
sequential steps regardless of length, and its number of fold rows grows with length, so the
greedy longest-first assignment balances rows per rank.
"""
import numpy as np


def fold_rows(n_frames, target, overlap, hop=200):
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


def infer_waveforms(mels, vocode_fn, target, overlap, hop=200, device=None):
    """Vocode a list of mels across the ranks of the default process group.

    ``vocode_fn(list_of_mels) -> list_of_f64_waveforms`` runs on this rank (the GPU model's
    ``generate_batch`` in production). Every rank receives the full list of waveforms in the
    input order. Waveform lengths are known from the mel lengths, so the gather is one
    fixed-size all-gather of padded float64 tensors.
    """
    import torch
    import torch.distributed as dist
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    frames = [int(m.shape[-1]) for m in mels]
    plan = shard(frames, world, target, overlap, hop)
    mine = plan[rank]
    wavs = vocode_fn([mels[i] for i in mine]) if mine else []
    if world == 1:
        return wavs
    lens = [(t - 1) * hop for t in frames]
    slots = max(len(p) for p in plan)
    width = max(lens)
    dev = device if device is not None else torch.device('cpu')
    buf = torch.zeros((slots, width), dtype=torch.float64, device=dev)
    for j, w in enumerate(wavs):
        buf[j, :len(w)] = torch.from_numpy(np.asarray(w, dtype=np.float64))
    bufs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf)
    out = [None] * len(mels)
    for r in range(world):
        host = bufs[r].cpu().numpy()
        for j, i in enumerate(plan[r]):
            out[i] = host[j, :lens[i]].copy()
    return out
