"""GPU parity at the BASELINE.json headline sizes (not just the tiny fixtures).

The oracle restatement (pinned bit-exact to the real reference by tests/test_oracle_golden.py)
runs the same workload on the host with the same Philox noise (seed, stream) and the HIP path
must reproduce it:

* C2  -- configs[1]: one 1000-frame mel, fatchord RAW 9-bit, target 11000 / overlap 550
        (18 folds incl. the zero-padded tail fold x 12,100 steps, 217,800 draws). Labels and the
        f64 waveform bit-exact. Run through the bench's path (generate_batch_device: one
        persistent launch of all 12,100 steps, no progress callback) and through the drop-in
        host API (WaveRNN.generate with the reference's progress callback).
* C3  -- configs[2]: the same mel in MOL mode; per-fold samples and waveform within 1e-4 RMS.
* C4  -- the per-GPU shape of configs[3]: 8 x 1000-frame mels in one call (144 fold rows; the
        persistent engine's row batches), utterances from the first and the last row batch
        against the oracle, every label.
* runtimeracer RAW 9-bit at the C2 shape.

Reference: vocoder/models/fatchord_version.py:155-259, runtimeracer_version.py:199-314,
vocoder/inference.py:59-95. Tolerances: BASELINE.json north_star (bit-exact 9-bit labels,
1e-4 RMS for MoL).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MOL_RMS_TOL = 1e-4
TARGET, OVERLAP, FRAMES = 11000, 550, 1000
NOISE_SEED = 1234


def first_divergence(a, b):
    d = np.argwhere(a != b)
    return None if len(d) == 0 else tuple(int(v) for v in d[np.argmin(d[:, 1])])


def make(model_type='fatchord-wavernn', mode='RAW', bits=9, weight_seed=0):
    from wavernn_amd.base import hparams_for
    from wavernn_amd.hparams import sp
    from wavernn_amd.model import WaveRNN
    from wavernn_amd.synth import synth_state_dict
    hp = hparams_for(model_type).copy(bits=bits, mode=mode)
    sd = synth_state_dict(hp, model_type, seed=weight_seed)
    m = WaveRNN(hp.rnn_dims, hp.fc_dims, hp.bits, hp.pad, hp.upsample_factors, sp.num_mels,
                hp.compute_dims, hp.res_out_dims, hp.res_blocks, sp.hop_size, sp.sample_rate,
                mode=hp.mode, model_type=model_type, device=0)
    m.load_state_dict(sd)
    return m, hp, sd


def oracle(sd, hp, model_type, mel_seed, stream=0):
    import torch
    from oracle.wavernn_oracle import oracle_infer_waveform
    from wavernn_amd.synth import synth_mel
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    return oracle_infer_waveform(sd, hp, model_type, synth_mel(FRAMES, mel_seed), target=TARGET,
                                 overlap=OVERLAP, seed=NOISE_SEED, stream=stream)


def device_mels(seeds):
    import torch
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    return [torch.from_numpy((synth_mel(FRAMES, s) / sp.max_abs_value).astype(np.float32)).cuda()
            for s in seeds]


def test_c2_full_size_labels_and_wave_bit_exact():
    from wavernn_amd.hparams import sp
    m, hp, sd = make()
    m.set_seed(NOISE_SEED)
    wavs = m.generate_batch(device_mels([0]), True, TARGET, OVERLAP, hp.mu_law, sp.preemphasize)
    assert m.last_engine() == 'persist'
    lab = m.last_batch_rows
    ref = oracle(sd, hp, 'fatchord-wavernn', 0)
    assert lab.shape == ref['labels'].shape == (18, 12100)
    agree = float((lab == ref['labels']).mean())
    assert agree == 1.0, f'C2 label agreement {agree}, first divergence (row, step) ' \
                         f'{first_divergence(lab, ref["labels"])}'
    assert wavs[0].dtype == np.float64 and wavs[0].shape == ref['wav'].shape == (199800,)
    assert np.array_equal(wavs[0], ref['wav'])
    # determinism of the exchange protocol: a second identical call gives the same bits
    m.set_seed(NOISE_SEED)
    wavs2 = m.generate_batch(device_mels([0]), True, TARGET, OVERLAP, hp.mu_law, sp.preemphasize)
    assert np.array_equal(m.last_batch_rows, lab) and np.array_equal(wavs2[0], wavs[0])


def test_c2_drop_in_host_api_with_reference_callback():
    """WaveRNN.generate on a host mel with the reference's progress callback: callbacks at
    i = 0, 100, ..., 12000 (fatchord_version.py:234-236), and the same bits as the oracle."""
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    m, hp, sd = make()
    m.set_seed(NOISE_SEED)
    calls = []
    wav = m.generate((synth_mel(FRAMES, 0) / sp.max_abs_value)[None], True, TARGET, OVERLAP,
                     hp.mu_law, sp.preemphasize,
                     progress_callback=lambda i, sl, b, r: calls.append((i, sl, b, r)))
    assert m.last_engine() == 'persist'
    assert [c[0] for c in calls] == list(range(0, 12100, 100))
    assert all(c[1] == 12100 and c[2] == 18 and c[3] > 0 for c in calls)
    ref = oracle(sd, hp, 'fatchord-wavernn', 0)
    assert np.array_equal(m.last_labels, ref['labels']), \
        f'first divergence {first_divergence(m.last_labels, ref["labels"])}'
    assert np.array_equal(wav, ref['wav'])


def test_c3_full_size_mol_within_tolerance():
    from wavernn_amd.hparams import sp
    m, hp, sd = make(mode='MOL')
    m.set_seed(NOISE_SEED)
    wavs = m.generate_batch(device_mels([0]), True, TARGET, OVERLAP, hp.mu_law, sp.preemphasize)
    assert m.last_engine() == 'persist'
    got = m.last_batch_rows.astype(np.float64)
    ref = oracle(sd, hp, 'fatchord-wavernn', 0)
    assert got.shape == ref['samples'].shape == (18, 12100)
    rms = float(np.sqrt(np.mean((got - ref['samples']) ** 2)))
    rms_w = float(np.sqrt(np.mean((wavs[0] - ref['wav']) ** 2)))
    assert rms <= MOL_RMS_TOL, f'C3 per-fold sample RMS {rms}'
    assert rms_w <= MOL_RMS_TOL, f'C3 waveform RMS {rms_w}'


def test_c4_per_gpu_shape_144_rows():
    """8 utterances x 18 folds = 144 rows in one generate_batch_device call; utterance u uses
    noise stream u. The first and the last utterance (first and last row batch) vs the oracle."""
    m, hp, sd = make()
    m.set_seed(NOISE_SEED)
    out, roff, S = m.generate_batch_device(device_mels(range(8)), True, TARGET, OVERLAP)
    assert m.last_engine() == 'persist'
    assert roff == [18 * u for u in range(9)] and S == 12100
    lab = out.cpu().numpy()
    for u in (0, 7):
        ref = oracle(sd, hp, 'fatchord-wavernn', u, stream=u)
        got = lab[roff[u]:roff[u + 1]]
        assert np.array_equal(got, ref['labels']), \
            f'utt {u}: first divergence (row, step) {first_divergence(got, ref["labels"])}'


def test_runtimeracer_c2_shape_bit_exact():
    m, hp, sd = make(model_type='runtimeracer-wavernn', weight_seed=4)
    m.set_seed(NOISE_SEED)
    out, roff, S = m.generate_batch_device(device_mels([0]), True, TARGET, OVERLAP)
    assert m.last_engine() == 'persist'
    lab = out.cpu().numpy()
    ref = oracle(sd, hp, 'runtimeracer-wavernn', 0)
    assert np.array_equal(lab, ref['labels']), \
        f'first divergence (row, step) {first_divergence(lab, ref["labels"])}'
