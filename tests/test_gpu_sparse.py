"""GPU: block-sparse execution of pruned checkpoints (VERDICT r5 missing #1).

The fork's Pruner (vocoder/pruner.py:60-88, target 0.90 in 1 x 4 groups, config/hparams.py:
266-270) leaves trained weights with 90 % of their 1 x 4 column blocks zero. The sparse
k_persist instances keep only the live blocks (LDS lists, kernels_persist.hip sp_products) and
accumulate them in the dense kernel's order, so:

* on the reference-made pruned fixtures (tests/golden/gen_golden.py: the reference's own
  Pruner masks, checked against wavernn_amd.prune) the labels and the f64 waveform are
  bit-exact (RAW) / within 1e-4 RMS (MOL), with the sparse instances running (sparse_info);
* the sparse launch equals the dense launch on the same weights bit for bit: labels, samples
  and the teacher-forced logits at the recorded steps (WRNN_SPARSE=0 runs the dense kernel);
* every rows-per-group variant (1-4) and the rotated launches, and a pruned libwavernn .bin
  through the chunked Vocoder path, run sparse with the same results as dense.
"""
import numpy as np
import pytest

from conftest import golden_case, golden_meta, is_continuous, wave_equal

pytestmark = pytest.mark.gpu

PRUNED = sorted(k for k, v in golden_meta().items() if v.get('prune'))
# the sparse instances are fatchord k_persist ones; a pruned runtimeracer model runs its dense
# kernels (test_pruned_fixture_matches_reference_on_the_sparse_path)
PRUNED_FAT = [k for k in PRUNED if golden_meta()[k]['model_type'] == 'fatchord-wavernn']


def _run(name, monkeypatch, sparse=True, debug_steps=None, nr_max=None):
    from test_gpu_parity import make_model
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    meta, gold = golden_case(name)
    monkeypatch.setenv('WRNN_SPARSE', '1' if sparse else '0')
    if nr_max:
        monkeypatch.setenv('WRNN_PERSIST_NR_MAX', str(nr_max))
    else:
        monkeypatch.delenv('WRNN_PERSIST_NR_MAX', raising=False)
    m, hp, sd = make_model(meta)
    m.set_engine('persist')
    if debug_steps:
        m.set_debug_steps(debug_steps)
    mel = synth_mel(meta['n_frames'], meta['mel_seed']) / sp.max_abs_value
    wav = m.generate(mel[None], meta['batched'], meta['target'], meta['overlap'], hp.mu_law,
                     sp.preemphasize, progress_callback=lambda *a: None)
    return meta, gold, m, wav


def test_pruned_fixtures_exist():
    assert len(PRUNED) >= 4, PRUNED


@pytest.mark.parametrize('name', PRUNED)
def test_pruned_fixture_matches_reference_on_the_sparse_path(name, monkeypatch):
    meta, gold, m, wav = _run(name, monkeypatch)
    info = m.sparse_info()
    if meta['model_type'] == 'fatchord-wavernn':
        assert info['available'] and info['last_call'], info
        assert info['density'] < 0.2, info
    else:  # no sparse instances for this topology: forced sparse runs its dense kernels
        assert not info['last_call'], info
    if is_continuous(meta):
        s = m.last_samples
        assert float(np.sqrt(np.mean((s.astype(np.float64) - gold['samples']) ** 2))) <= 1e-4
        assert float(np.sqrt(np.mean((wav - gold['wav']) ** 2))) <= 1e-4
        return
    lab = m.last_labels
    assert lab.shape == gold['labels'].shape
    if meta.get('gru_scale', 1.0) != 1.0:
        # trained-like statistics: the near-tie gate with its measured allowance
        # (tests/test_gpu_trained.py, kind 'sparse')
        from test_gpu_trained import near_tie_gate
        near_tie_gate(name, 'sparse', meta, gold, lab, wav,
                      lambda steps: _run(name, monkeypatch, debug_steps=steps)[2])
        return
    d = np.argwhere(lab != gold['labels'])
    assert len(d) == 0, f'{name}: first divergence (row, step) {d[np.argmin(d[:, 1])] if len(d) else None}'
    assert wave_equal(wav, gold)


@pytest.mark.parametrize('name', PRUNED_FAT)
def test_sparse_equals_dense_bit_for_bit(name, monkeypatch):
    """Same weights, sparse vs dense k_persist (same plan): identical labels / samples and
    identical teacher-forced logits (the sparse sums skip only exact-zero products)."""
    meta, gold = golden_case(name)
    steps = [int(s) for s in gold['logits_steps']][:4]
    _, _, ms, _ = _run(name, monkeypatch, sparse=True, debug_steps=steps)
    _, _, md, _ = _run(name, monkeypatch, sparse=False, debug_steps=steps)
    assert ms.sparse_info()['last_call'] and not md.sparse_info()['last_call']
    assert ms.plan_info() == md.plan_info()
    if is_continuous(meta):
        assert np.array_equal(ms.last_samples.view(np.uint32), md.last_samples.view(np.uint32))
    else:
        assert np.array_equal(ms.last_labels, md.last_labels)
    rows = range(meta['num_folds'])
    for s in steps:
        a, b = ms.debug_logits(s, rows), md.debug_logits(s, rows)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), f'step {s}'
        # and the logit gate against the reference's own logits
        ref = gold['logits'][list(gold['logits_steps']).index(s)]
        err = float(np.abs(a.astype(np.float64) - ref).max())
        assert err <= 1e-5 * max(1.0, float(np.abs(ref).max())), (s, err)


@pytest.mark.parametrize('nr', [1, 2, 3, 4])
def test_sparse_rows_per_group_variants_equal_dense(nr, monkeypatch):
    """The 10-bit default shape (9 rows, 1024 classes: the 32-class slot lists) at every row
    count per group, sparse vs dense -- identical labels."""
    name = 'fatchord_raw10_pruned_defaults'
    meta, gold, ms, _ = _run(name, monkeypatch, sparse=True, nr_max=nr)
    assert ms.sparse_info()['last_call']
    assert all(L[1] == nr for L in ms.plan_info()), ms.plan_info()
    _, _, md, _ = _run(name, monkeypatch, sparse=False, nr_max=nr)
    assert np.array_equal(ms.last_labels, md.last_labels)
    assert np.array_equal(ms.last_labels, gold['labels'])


def test_sparse_rotation_runs_at_c2_shape(monkeypatch):
    """C2's 18 rows: the rotated sparse launches (3 rows / 2 rows per group)."""
    meta, gold, m, wav = _run('fatchord_raw9_c2_pruned', monkeypatch)
    assert m.sparse_info()['last_call']
    assert m.rot_info()[0] >= 2, m.rot_info()
    assert np.array_equal(m.last_labels, gold['labels'])


def test_pruned_bin_through_the_vocoder_runs_sparse(tmp_path, monkeypatch):
    """A 90 %-pruned fatchord .bin (the reference Pruner's masks) through the libwavernn chunked
    path: the sparse image is built from the file's zero blocks, and every chunk's labels equal
    the oracle's unbatched generate of that chunk."""
    import torch
    from oracle.wavernn_oracle import oracle_infer_waveform
    from wavernn_amd import convert
    from wavernn_amd.base import hparams_for
    from wavernn_amd.hparams import sp
    from wavernn_amd.libwavernn import Vocoder
    from wavernn_amd.prune import prune_state_dict
    from wavernn_amd.synth import synth_mel, synth_state_dict
    monkeypatch.setenv('WRNN_SPARSE', '1')
    mt = 'fatchord-wavernn'
    hp = hparams_for(mt)  # the fork default (10 bits): what the Vocoder builds
    sd = prune_state_dict(synth_state_dict(hp, mt, seed=45), mt, z=0.9)
    path = tmp_path / 'voc.bin'
    with open(path, 'wb') as f:
        convert.write_bin(f, sd, hp, mt)
    v = Vocoder(str(path), mt, verbose=False)
    v.setRandomSeed(23)
    v.load(max_threads=3)
    m = v._model
    assert m.sparse_info()['available']
    mel = synth_mel(40, 10)
    wav = v.vocode_mel(mel.copy())
    assert np.isfinite(wav).all()
    hp_w = hparams_for(mt)
    wave_len = mel.shape[1] * sp.hop_size
    tgt = max(hp_w.gen_target, int(np.ceil((wave_len - hp_w.gen_overlap) / 3 - hp_w.gen_overlap)))
    chunks = v.fold_mel_with_overlap(mel / sp.max_abs_value, tgt, hp_w.gen_overlap)
    m.set_seed(23)
    dev = [torch.from_numpy(np.ascontiguousarray(c, np.float32)).cuda() for c in chunks]
    lab, roff, S = m.generate_batch_device(dev, False, 0, 0)
    assert m.sparse_info()['last_call']
    lab = lab.cpu().numpy()
    for u, c in enumerate(chunks):
        ref = oracle_infer_waveform(sd, hp, mt, c * sp.max_abs_value, batched=False, seed=23, stream=u)
        assert np.array_equal(lab[roff[u]:roff[u + 1]], ref['labels']), f'chunk {u}'


def test_sparse_image_absent_for_dense_weights(monkeypatch):
    from test_gpu_parity import make_model
    meta, _ = golden_case('fatchord_raw9_tiny')
    m, _, _ = make_model(meta)
    info = m.sparse_info()
    assert not info['available'] and info['density'] == 1.0, info


def test_half_pruned_weights_fall_back_to_dense(monkeypatch):
    """50 % live blocks do not fit the LDS lists: no sparse image, the dense kernel runs them."""
    from test_libwavernn import pruned_state_dict
    from wavernn_amd.base import hparams_for
    from wavernn_amd.model import WaveRNN
    from wavernn_amd.hparams import sp
    hp = hparams_for('fatchord-wavernn').copy(bits=9)
    sd = pruned_state_dict(hp, 'fatchord-wavernn', keep=0.5)
    m = WaveRNN(hp.rnn_dims, hp.fc_dims, hp.bits, hp.pad, hp.upsample_factors, sp.num_mels,
                hp.compute_dims, hp.res_out_dims, hp.res_blocks, sp.hop_size, sp.sample_rate,
                mode=hp.mode, model_type='fatchord-wavernn', device=0)
    m.load_state_dict(sd)
    assert not m.sparse_info()['available']
