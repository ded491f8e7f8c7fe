"""libwavernn backend: the .bin weight format and the chunked host path.

CPU only: the .bin reader of the C-ABI (``wrnn_bin_read``, host code) against the writer on
dense and 1x4-pruned weights of both topologies, its error behaviour, and the host side of
``Vocoder.vocode_mel`` (fold, cross-fade, mu-law, de-emphasis, fade-out) against fixtures
recorded from the reference's own ``vocoder/libwavernn/inference.py``
(tests/golden/gen_libwavernn_golden.py) with the same deterministic per-chunk stand-in.
"""
import io
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN

sys.path.insert(0, GOLDEN)
from gen_libwavernn_golden import CASES, fake_mel_to_wav  # noqa: E402


def pruned_state_dict(hp, model_type, seed=3, keep=0.5):
    from wavernn_amd.synth import synth_state_dict
    rng = np.random.default_rng(seed)
    sd = {}
    for k, v in synth_state_dict(hp, model_type, seed=seed).items():
        v = np.array(v, dtype=np.float32)
        if v.ndim == 2 and (k.startswith(('rnn', 'fc', 'I.'))):
            r, c = v.shape
            v = v * np.repeat(rng.random((r, c // 4)) < keep, 4, axis=1)
        sd[k] = v
    return sd


TOPOLOGIES = [('fatchord-wavernn', 9), ('runtimeracer-wavernn', 10), ('geneing-wavernn', 10)]


@pytest.mark.parametrize('model_type,bits', TOPOLOGIES)
@pytest.mark.parametrize('keep', [1.0, 0.3])
def test_bin_round_trip(model_type, bits, keep):
    from wavernn_amd import convert
    from wavernn_amd.base import hparams_for
    hp = hparams_for(model_type).copy(bits=bits)
    sd = pruned_state_dict(hp, model_type, keep=keep)
    f = io.BytesIO()
    convert.write_bin(f, sd, hp, model_type)
    back = convert.read_bin(f.getvalue(), hp, model_type)
    want = {k: v for k, v in sd.items() if k != 'step' and not k.endswith('num_batches_tracked')}
    assert set(back) == set(want)
    for k, v in want.items():
        assert back[k].shape == v.shape, k
        assert np.array_equal(back[k], v), k


@pytest.mark.parametrize('model_type,bits', TOPOLOGIES)
def test_bin_fp16_round_trip(model_type, bits):
    """elSize 2 (convert.py:12 'change to 2 for fp16', wavernn.cpp:98): binary16 arrays, widened
    exactly to fp32 on load -- every tensor equals the state dict rounded to fp16; BatchNorm eps
    stays fp32. The file is half the size of the fp32 one (plus headers / index streams)."""
    from wavernn_amd import convert
    from wavernn_amd.base import hparams_for
    hp = hparams_for(model_type).copy(bits=bits)
    sd = pruned_state_dict(hp, model_type, keep=0.5)
    f16, f32 = io.BytesIO(), io.BytesIO()
    convert.write_bin(f16, sd, hp, model_type, el_size=2)
    convert.write_bin(f32, sd, hp, model_type)
    assert len(f16.getvalue()) < 0.6 * len(f32.getvalue())
    back = convert.read_bin(f16.getvalue(), hp, model_type)
    for k, v in sd.items():
        if k == 'step' or k.endswith('num_batches_tracked'):
            continue
        assert np.array_equal(back[k], v.astype(np.float16).astype(np.float32)), k
    with pytest.raises(ValueError, match='el_size'):
        convert.write_bin(io.BytesIO(), sd, hp, model_type, el_size=8)


def test_half_widening_special_values():
    """Subnormal, signed zero, inf and the largest half through the reader's widening."""
    import struct
    from wavernn_amd import convert
    from wavernn_amd.base import hparams_for
    mt = 'geneing-wavernn'
    hp = hparams_for(mt).copy(bits=9, mode='BITS')
    sd = pruned_state_dict(hp, mt, keep=1.0)
    vals = np.array([6e-8, -6e-8, 2.0 ** -14, -0.0, 65504.0, np.inf, -np.inf, 1 / 3], np.float32)
    sd['upsample.up_layers.1.weight'] = np.resize(vals, sd['upsample.up_layers.1.weight'].shape)
    f = io.BytesIO()
    convert.write_bin(f, sd, hp, mt, el_size=2)
    got = convert.read_bin(f.getvalue(), hp, mt)['upsample.up_layers.1.weight'].reshape(-1)
    want = np.resize(vals, got.shape).astype(np.float16).astype(np.float32)
    assert np.array_equal(got, want) and np.signbit(got[3]) and got[0] > 0


def test_compress_format():
    """convert.py:60-74 on a hand-made matrix: kept blocks row by row, 255 row ends + 1."""
    from wavernn_amd.convert import compress
    W = np.zeros((2, 12), np.float32)
    W[0, 5] = 1.5           # block 1 of row 0
    W[1, 0:4] = [1, 2, 3, 4]  # block 0 of row 1
    W[1, 11] = -2           # block 2 of row 1
    w, idx = compress(W)
    assert idx.tolist() == [1, 255, 0, 2, 255, 255]
    assert w.tolist() == [0, 1.5, 0, 0, 1, 2, 3, 4, 0, 0, 0, -2]


def test_bin_errors():
    import struct
    from wavernn_amd import convert
    from wavernn_amd.base import hparams_for
    mt = 'runtimeracer-wavernn'
    hp = hparams_for(mt).copy(bits=9, mode='RAW')
    f = io.BytesIO()
    convert.write_bin(f, pruned_state_dict(hp, mt), hp, mt)
    data = f.getvalue()
    with pytest.raises(ValueError, match='truncated|bad array'):
        convert.read_bin(data[:len(data) // 2], hp, mt)
    with pytest.raises(ValueError, match='trailing'):
        convert.read_bin(data + b'\0' * 8, hp, mt)
    with pytest.raises(ValueError, match='does not match'):  # 10-bit model, 9-bit file
        convert.read_bin(data, hparams_for(mt).copy(bits=10, mode='RAW'), mt)
    with pytest.raises(ValueError, match='Cannot open file'):
        convert.read_bin(b'\1\2', hp, mt)
    bad = bytearray(data)
    bad[16 + 68:16 + 72] = struct.pack('@i', 8)  # elSize of the first layer
    with pytest.raises(ValueError, match='elSize 8'):
        convert.read_bin(bytes(bad), hp, mt)
    with pytest.raises(ValueError, match='does not match'):  # fatchord reader, runtimeracer file
        convert.read_bin(data, hparams_for('fatchord-wavernn').copy(bits=9, mode='RAW'),
                         'fatchord-wavernn')


def _fake_vocoder(model_type, n_chunks):
    from wavernn_amd.libwavernn import Vocoder
    v = Vocoder('unused.bin', model_type, verbose=False)
    v._model = object()  # loaded (no device needed for the host path)
    v._n_chunks = n_chunks
    v._vocode_chunks = lambda chunks, cb=None: [fake_mel_to_wav(c) for c in chunks]
    return v


@pytest.mark.parametrize('name', sorted(CASES))
def test_vocode_mel_host_path_matches_reference(name):
    g = np.load(os.path.join(GOLDEN, f'libwavernn_{name}.npz'))
    model_type, T, nw, seed = CASES[name]
    v = _fake_vocoder(model_type, nw)
    wav = v.vocode_mel(g['mel'].copy(), normalize=True)
    assert wav.dtype == g['wav'].dtype and wav.shape == g['wav'].shape
    assert np.array_equal(wav, g['wav'])
    folded = v.fold_mel_with_overlap(g['mel'] / 4.0, 2750, 1000)
    assert np.array_equal(np.stack(folded), g['folded'])
    assert np.array_equal(v.unfold_wav_with_overlap(g['fw'].copy(), 1000, 500), g['unfolded'])


def test_vocoder_requires_load():
    from wavernn_amd.libwavernn import Vocoder
    v = Vocoder('unused.bin', 'runtimeracer-wavernn', verbose=False)
    with pytest.raises(RuntimeError, match='No processing thread wrappers'):
        v.vocode_mel(np.zeros((80, 10), np.float32))
