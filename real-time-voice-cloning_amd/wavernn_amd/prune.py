"""Block-sparse pruning masks of the reference's training-time Pruner (host side, torch-CPU).

The fork trains with ``vocoder/pruner.py`` when ``use_sparsification`` is set
(``config/hparams.py:265-270``: target 0.90, groups of 4; ``vocoder/models/base.py:46-48``
builds the Pruner over ``model.prune_layers``). A pruned checkpoint stores its weights with the
masks already applied (``PruneMask.apply_mask``, pruner.py:55-58), so loading one needs nothing
from here: the runtime finds the zero 1x4 blocks itself (``csrc/runtime.hip`` pack_persist_sparse).
This module restates the mask so tests and the bench can prune the seeded synthetic weights
exactly as the reference would; ``tests/golden/gen_golden.py`` checks it against the
reference's own Pruner.

Restated (same torch ops, so the same float32 group sums and the same sort):
* ``PruneMask.mask_from_matrix`` (pruner.py:60-88): per gate matrix (GRU weights split in 3),
  the L1 norm of each 1 x ``group`` column block, the ``int(rows * cols // group * z)``-th
  smallest as the threshold, blocks >= threshold kept;
* ``PruneMask.init_mask`` / ``get_params`` (pruner.py:21-47): Linear -> ``weight``; GRU ->
  ``weight_ih_l0`` and ``weight_hh_l0`` (``prune_rnn_input=True``, pruner.py:97);
* ``prune_layers`` per topology: fatchord_version.py:115, runtimeracer_version.py:134,
  geneing_version.py:116.
"""
import numpy as np

PRUNE_LAYERS = {
    'fatchord-wavernn': ['I', 'rnn1', 'rnn2', 'fc1', 'fc2', 'fc3'],
    'runtimeracer-wavernn': ['I', 'rnn1', 'rnn2', 'rnn3', 'rnn4', 'fc1', 'fc2', 'fc3', 'fc4', 'fc5'],
    'geneing-wavernn': ['I', 'rnn1', 'fc1', 'fc3'],
}


def mask_from_matrix(W, z, group, splits):
    """pruner.py:60-88 on one parameter matrix W (rows, cols); `splits` gate matrices."""
    import torch
    W = torch.as_tensor(W)
    split = W.size(0) // splits
    parts = torch.split(W, split) if split > 1 else W
    out = []
    for P in parts:
        N = P.shape[1]
        S = torch.abs(P).reshape(P.shape[0], N // group, group).sum(dim=2)
        sorted_abs, _ = torch.sort(S.view(-1))
        k = int(P.shape[0] * P.shape[1] // group * z)
        mask = (S >= sorted_abs[k]).float()
        out.append(mask.unsqueeze(2).expand(-1, -1, group).reshape(P.shape[0], P.shape[1]))
    return torch.cat(out)


def prune_state_dict(sd, model_type, z=0.9, group=4):
    """A copy of `sd` with the Pruner's masks at sparsity `z` applied to every pruned layer
    (what a checkpoint trained past start_prune + prune_steps carries)."""
    import torch
    out = dict(sd)
    for layer in PRUNE_LAYERS[model_type]:
        names = ([f'{layer}.weight_ih_l0', f'{layer}.weight_hh_l0'] if layer.startswith('rnn')
                 else [f'{layer}.weight'])
        for n in names:
            W = torch.from_numpy(np.ascontiguousarray(np.asarray(sd[n], dtype=np.float32)))
            M = mask_from_matrix(W, z, group, 3 if layer.startswith('rnn') else 1)
            out[n] = (W * M).numpy()
    return out


def block_density(sd, model_type, group=4):
    """Fraction of nonzero 1 x group blocks over the pruned layers' matrices."""
    live = total = 0
    for layer in PRUNE_LAYERS[model_type]:
        names = ([f'{layer}.weight_ih_l0', f'{layer}.weight_hh_l0'] if layer.startswith('rnn')
                 else [f'{layer}.weight'])
        for n in names:
            W = np.asarray(sd[n])
            b = np.abs(W.reshape(W.shape[0], -1, group)).sum(axis=2) != 0
            live += int(b.sum())
            total += b.size
    return live / max(total, 1)
