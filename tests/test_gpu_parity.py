"""GPU parity: the HIP path (through the C-ABI) against the reference's golden outputs and the
oracle restatement. Bar (BASELINE.json north_star): RAW 9/10-bit labels bit-exact, waveform
bit-exact (f64 post-processing is the reference's own numpy/scipy code); MOL and geneing 'RAW'
(Beta) float paths within 1e-4 RMS.
"""
import numpy as np
import pytest

from conftest import golden_case, golden_meta, hparams_of, is_continuous

pytestmark = pytest.mark.gpu

MOL_RMS_TOL = 1e-4


def make_model(meta):
    from wavernn_amd.model import WaveRNN
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_state_dict
    hp = hparams_of(meta)
    sd = synth_state_dict(hp, meta['model_type'], seed=meta['weight_seed'],
                          logit_scale=meta['logit_scale'])
    m = WaveRNN(hp.rnn_dims, hp.fc_dims, hp.bits, hp.pad, hp.upsample_factors, sp.num_mels,
                hp.compute_dims, hp.res_out_dims, hp.res_blocks, sp.hop_size, sp.sample_rate,
                mode=hp.mode, model_type=meta['model_type'], device=0)
    m.load_state_dict(sd)
    m.set_seed(meta['noise_seed'])
    return m, hp, sd


def run_case(name, engine='auto'):
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    meta, gold = golden_case(name)
    m, hp, sd = make_model(meta)
    m.set_engine(engine)
    mel = synth_mel(meta['n_frames'], meta['mel_seed']) / sp.max_abs_value
    wav = m.generate(mel[None], meta['batched'], meta['target'], meta['overlap'], hp.mu_law,
                     sp.preemphasize, progress_callback=lambda *a: None)
    if engine != 'auto':
        assert m.last_engine() == engine
    return meta, gold, m, wav


def first_divergence(a, b):
    d = np.argwhere(a != b)
    return None if len(d) == 0 else tuple(d[np.argmin(d[:, 1])])


def engine_cases(continuous):
    # both engines run every topology (PERSIST: kernels_persist.hip fatchord,
    # kernels_persist_rr.hip runtimeracer, kernels_persist_gen.hip geneing)
    out = []
    for k, v in golden_meta().items():
        if is_continuous(v) != continuous:
            continue
        out.append((k, 'chain'))
        out.append((k, 'persist'))
    return out


RAW_CASES = engine_cases(False)  # RAW and geneing 'BITS': categorical over 2**bits classes
MOL_CASES = engine_cases(True)   # MOL and geneing 'RAW' (Beta): float samples


@pytest.mark.parametrize('name,engine', RAW_CASES)
def test_raw_labels_and_wave_bit_exact(name, engine):
    meta, gold, m, wav = run_case(name, engine)
    lab = m.last_labels
    assert lab.shape == gold['labels'].shape == (meta['num_folds'], meta['seq_len'])
    agree = float((lab == gold['labels']).mean())
    assert agree == 1.0, f'{name}/{engine}: label agreement {agree}, first divergence (row, step) ' \
                         f'{first_divergence(lab, gold["labels"])}'
    assert wav.dtype == np.float64 and wav.shape == gold['wav'].shape
    assert np.array_equal(wav, gold['wav'])


@pytest.mark.parametrize('name,engine', MOL_CASES)
def test_mol_float_path_within_tolerance(name, engine):
    meta, gold, m, wav = run_case(name, engine)
    s = m.last_samples
    rms = float(np.sqrt(np.mean((s.astype(np.float64) - gold['samples']) ** 2)))
    rms_w = float(np.sqrt(np.mean((wav - gold['wav']) ** 2)))
    assert rms <= MOL_RMS_TOL, f'{name}: per-fold sample RMS {rms}'
    assert rms_w <= MOL_RMS_TOL, f'{name}: waveform RMS {rms_w}'


def test_noise_matches_philox_contract():
    from oracle import philox
    meta, gold, m, wav = run_case('fatchord_raw9_tiny')
    B = meta['num_folds']
    n_steps = 64
    q = m.debug_noise(n_steps, B)
    ref = philox.raw_exp_noise(meta['noise_seed'], 0, np.arange(n_steps), np.arange(B), m.n_classes)
    assert np.array_equal(q, ref)


def test_upsample_network_matches_oracle():
    import torch
    from oracle.wavernn_oracle import OracleWaveRNN
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    meta, gold, m, wav = run_case('fatchord_raw9_tiny')
    T = meta['n_frames']
    mel_up, aux = m.debug_upsample(T)
    hp = hparams_of(meta)
    from wavernn_amd.synth import synth_state_dict
    sd = synth_state_dict(hp, meta['model_type'], seed=meta['weight_seed'])
    o = OracleWaveRNN(sd, hp, meta['model_type'])
    mel = torch.from_numpy(synth_mel(T, meta['mel_seed'])[None] / sp.max_abs_value)
    with torch.no_grad():
        padded = o.pad_tensor(mel.transpose(1, 2), pad=hp.pad, side='both').transpose(1, 2)
        ref_aux = o.resnet(padded)[0].numpy()
        ref_mel, _ = o.upsample(padded)
    ref_mel = ref_mel[0].numpy().T
    np.testing.assert_allclose(aux, ref_aux, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(mel_up, ref_mel, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize('case', ['fatchord_raw9_sharp_tiny', 'runtimeracer_raw9_tiny',
                                  'geneing_bits10_tiny'])
@pytest.mark.parametrize('n_utts', [3, 4, 6, 10])
def test_persist_multi_row_groups_match_oracle(n_utts, case):
    """5 fold rows per utterance -> 15 / 20 / 30 / 50 rows: 2 and 3 rows per XCD group (the
    padded-row variants of the persistent engine) and, past 24 rows, consecutive launches over
    row batches (30 rows -> 2 batches of 2 rows per group, 50 -> 3 batches of 3), every row
    against the oracle."""
    import torch
    from oracle.wavernn_oracle import oracle_infer_waveform
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    meta, _ = golden_case(case)
    m, hp, sd = make_model(meta)
    mels = [synth_mel(meta['n_frames'], 100 + u) / sp.max_abs_value for u in range(n_utts)]
    dev = [torch.from_numpy(x.astype(np.float32)).cuda() for x in mels]
    m.set_engine('persist')
    m.set_seed(meta['noise_seed'])
    try:
        lab, row_off, S = m.generate_batch_device(dev, True, meta['target'], meta['overlap'])
    except ValueError as e:  # no spill-free variant for this row count on this build
        pytest.skip(str(e))
    assert m.last_engine() == 'persist'
    lab = lab.cpu().numpy()
    for u in range(n_utts):
        ref = oracle_infer_waveform(sd, hp, meta['model_type'], mels[u] * sp.max_abs_value,
                                    target=meta['target'], overlap=meta['overlap'],
                                    seed=meta['noise_seed'], stream=u)
        got = lab[row_off[u]:row_off[u + 1]]
        assert np.array_equal(got, ref['labels']), \
            f'utt {u}: first divergence {first_divergence(got, ref["labels"])}'


@pytest.mark.parametrize('case', ['fatchord_mol_tiny', 'runtimeracer_mol_tiny', 'geneing_mol_tiny',
                                  'geneing_raw_beta_tiny'])
def test_persist_row_batches_mol_within_tolerance(case):
    """MOL / Beta float path over row batches (6 utterances x the case's fold rows)."""
    import torch
    from oracle.wavernn_oracle import oracle_infer_waveform
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    meta, _ = golden_case(case)
    m, hp, sd = make_model(meta)
    n_utts = 6
    mels = [synth_mel(meta['n_frames'], 200 + u) / sp.max_abs_value for u in range(n_utts)]
    dev = [torch.from_numpy(x.astype(np.float32)).cuda() for x in mels]
    m.set_engine('persist')
    m.set_seed(meta['noise_seed'])
    out, row_off, S = m.generate_batch_device(dev, True, meta['target'], meta['overlap'])
    assert m.last_engine() == 'persist'
    out = out.cpu().numpy()
    for u in range(n_utts):
        ref = oracle_infer_waveform(sd, hp, meta['model_type'], mels[u] * sp.max_abs_value,
                                    target=meta['target'], overlap=meta['overlap'],
                                    seed=meta['noise_seed'], stream=u)
        got = out[row_off[u]:row_off[u + 1]].astype(np.float64)
        rms = float(np.sqrt(np.mean((got - ref['samples']) ** 2)))
        assert rms <= MOL_RMS_TOL, f'utt {u}: per-fold sample RMS {rms}'
