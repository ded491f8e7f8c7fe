"""Host-side pieces of the drop-in (CPU only): hparams, synthetic weights vs the reference
state-dict layout, and the f64 post-processing restatement vs the oracle."""
import numpy as np
import pytest

from conftest import golden_case, hparams_of


def test_hparams_parse_and_values():
    from wavernn_amd.hparams import HParams, sp, wavernn_fatchord, wavernn_runtimeracer
    assert sp.hop_size == 200 and sp.sample_rate == 16000 and sp.max_abs_value == 4.
    assert wavernn_fatchord.gen_target == 3000 and wavernn_fatchord.gen_overlap == 1500
    assert wavernn_runtimeracer.gen_target == 6000 and wavernn_runtimeracer.rnn_dims == 256
    hp = HParams(a=1, b=(1, 2)).parse("a=3, c='x'")   # comma-separated, as the reference
    assert hp.a == 3 and hp.c == 'x' and hp.b == (1, 2)


@pytest.mark.parametrize('model_type', ['fatchord-wavernn', 'runtimeracer-wavernn'])
def test_synth_state_dict_is_deterministic_and_shaped(model_type):
    from wavernn_amd.hparams import wavernn_fatchord, wavernn_runtimeracer
    from wavernn_amd.synth import synth_state_dict, state_dict_spec
    hp = (wavernn_fatchord if model_type.startswith('fatchord') else wavernn_runtimeracer).copy(bits=9)
    a = synth_state_dict(hp, model_type, seed=3)
    b = synth_state_dict(hp, model_type, seed=3)
    spec = state_dict_spec(hp, model_type)
    for k, shape in spec.items():
        assert a[k].shape == shape and a[k].dtype == np.float32
        assert np.array_equal(a[k], b[k])
    # key set and shapes are also asserted against the live reference model by gen_golden.py
    assert 'rnn1.weight_ih_l0' in spec and 'upsample.up_layers.5.weight' in spec


def test_labels_to_samples_is_the_reference_fp32_formula():
    from wavernn_amd.audio import labels_to_samples
    meta, gold = golden_case('fatchord_raw9_tiny')
    import torch
    k = torch.from_numpy(gold['labels'].astype(np.int64))
    ref = (2 * k.float() / (512 - 1.) - 1.).numpy()     # fatchord_version.py:228
    assert np.array_equal(labels_to_samples(gold['labels'], 512), ref)


@pytest.mark.parametrize('name', ['fatchord_raw9_tiny', 'fatchord_mol_tiny',
                                  'fatchord_raw10_unbatched_tiny'])
def test_postprocess_matches_reference_waveform(name):
    """Given the reference's per-fold samples, the host post-processing reproduces the
    reference waveform bit for bit."""
    from wavernn_amd.audio import labels_to_samples, postprocess
    meta, gold = golden_case(name)
    n = 2 ** meta['bits'] if meta['mode'] == 'RAW' else 30
    smp = labels_to_samples(gold['labels'], n) if meta['mode'] == 'RAW' else gold['samples']
    hp = hparams_of(meta)
    wav = postprocess(smp, meta['batched'], meta['target'], meta['overlap'],
                      hp.mu_law if meta['mode'] == 'RAW' else False, True, n,
                      (meta['n_frames'] - 1) * 200, 200)
    assert np.array_equal(wav, gold['wav'])


@pytest.mark.parametrize('name', ['fatchord_raw9_tiny', 'fatchord_raw9_config1',
                                  'fatchord_raw10_defaults', 'runtimeracer_raw9_tiny'])
def test_fused_label_post_matches_reference_waveform(name):
    """The library's fused label post-processing (wrnn_post_overlaps / wrnn_post_assemble)
    reproduces the reference waveform of each batched RAW fixture bit for bit."""
    from wavernn_amd import _abi
    from wavernn_amd.audio import postprocess_labels
    meta, gold = golden_case(name)
    if not meta['batched'] or meta['mode'] != 'RAW':
        pytest.skip('fused path covers batched categorical rows')
    hp = hparams_of(meta)
    wav = postprocess_labels(gold['labels'], meta['target'], meta['overlap'], hp.mu_law, True,
                             2 ** meta['bits'], (meta['n_frames'] - 1) * 200, 200,
                             _abi.load_library())
    assert wav is not None
    assert np.array_equal(wav, gold['wav'])


def test_short_mel_raises_like_reference():
    """wave_len < 20*hop: the reference's fade-out broadcast fails (fatchord_version.py:255)."""
    from wavernn_amd.audio import postprocess
    with pytest.raises(ValueError):
        postprocess(np.zeros((1, 1200), np.float32), False, None, None, True, True, 512, 1000, 200)


def test_inference_api_surface():
    from wavernn_amd import inference
    assert not inference.is_loaded()
    with pytest.raises(Exception, match='Please load Wave-RNN'):
        inference.infer_waveform(np.zeros((80, 10), np.float32))
    with pytest.raises(NotImplementedError):
        inference.load_model('x.pt', voc_type='tensorflow')
    import vocoder.libwavernn.inference as lw   # libwavernn drop-in (voc_type='libwavernn')
    from wavernn_amd.libwavernn import Vocoder
    assert lw.Vocoder is Vocoder
    import vocoder.inference as drop_in   # the reference's module name resolves to ours
    assert drop_in.infer_waveform is inference.infer_waveform
