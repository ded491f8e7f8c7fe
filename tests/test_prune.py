"""wavernn_amd.prune: the reference Pruner's mask (vocoder/pruner.py:60-88) restated, host only.

The pruned golden fixtures (tests/golden/gen_golden.py) were made by the REFERENCE's Pruner and
checked there against this restatement bit for bit; test_oracle_golden.py then pins the oracle
on those weights against the reference's labels. Here: the mask's structure on every topology."""
import numpy as np
import pytest

TOPO = [('fatchord-wavernn', 9), ('runtimeracer-wavernn', 10), ('geneing-wavernn', 10)]


@pytest.mark.parametrize('mt,bits', TOPO)
@pytest.mark.parametrize('z', [0.5, 0.9])
def test_mask_structure(mt, bits, z):
    from wavernn_amd.base import hparams_for
    from wavernn_amd.prune import PRUNE_LAYERS, block_density, prune_state_dict
    from wavernn_amd.synth import synth_state_dict
    hp = hparams_for(mt).copy(bits=bits)
    sd = synth_state_dict(hp, mt, seed=3)
    pr = prune_state_dict(sd, mt, z=z)
    assert abs(block_density(pr, mt) - (1 - z)) < 2e-3
    for layer in PRUNE_LAYERS[mt]:
        names = ([f'{layer}.weight_ih_l0', f'{layer}.weight_hh_l0'] if layer.startswith('rnn')
                 else [f'{layer}.weight'])
        for n in names:
            W, P = np.asarray(sd[n]), np.asarray(pr[n])
            g = P.reshape(P.shape[0], -1, 4)
            live = (g != 0).any(axis=2)
            # whole 1 x 4 groups: a group is either untouched or all zero
            assert np.array_equal(np.where(live[..., None], W.reshape(g.shape), 0), g)
            # per gate matrix (GRU: 3 splits) the kept fraction is 1 - z (the k-th smallest
            # block norm is the threshold; ties at it are kept)
            splits = 3 if layer.startswith('rnn') else 1
            for part in np.split(live, splits, axis=0):
                assert part.mean() >= (1 - z) - 1e-9 and part.mean() < (1 - z) + 0.01
            # the kept blocks are the largest by L1 norm
            norms = np.abs(W.reshape(g.shape)).astype(np.float32).sum(axis=2)
            for pl, pn in zip(np.split(live, splits, axis=0), np.split(norms, splits, axis=0)):
                assert pn[pl].min() >= pn[~pl].max()
    # everything else untouched
    for k in sd:
        if not any(k.startswith(l + '.') for l in PRUNE_LAYERS[mt]) or 'bias' in k:
            assert np.array_equal(np.asarray(sd[k]), np.asarray(pr[k])), k
