"""GPU: libwavernn .bin weights and the chunked libwavernn path on the MI355X.

* a .bin file (dense or 1x4-pruned) loads to the same device model as the state dict it was
  written from: identical labels, both topologies;
* ``wavernn_amd.libwavernn.Vocoder`` vocodes the raw-mel chunks as one unbatched multi-row
  call; every chunk's labels equal the oracle's unbatched generate of that chunk (noise stream =
  chunk index), and ``vocode_mel`` returns the reference's wave length.
"""
import io

import numpy as np
import pytest

from test_libwavernn import pruned_state_dict

pytestmark = pytest.mark.gpu


def _model(hp, mt):
    from wavernn_amd.base import init_voc_model
    from wavernn_amd.hparams import sp  # noqa: F401
    m, _ = init_voc_model(mt, 0, override_hp_fatchord=hp, override_hp_runtimeracer=hp,
                          override_hp_geneing=hp)
    return m


@pytest.mark.parametrize('mt,bits', [('fatchord-wavernn', 9), ('runtimeracer-wavernn', 10),
                                     ('geneing-wavernn', 10)])
@pytest.mark.parametrize('keep', [1.0, 0.3])
def test_bin_loaded_model_equals_state_dict_model(mt, bits, keep):
    from wavernn_amd import convert
    from wavernn_amd.base import hparams_for
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    hp = hparams_for(mt).copy(bits=bits)
    sd = pruned_state_dict(hp, mt, keep=keep)
    f = io.BytesIO()
    convert.write_bin(f, sd, hp, mt)
    a, b = _model(hp, mt), _model(hp, mt)
    a.load_state_dict(sd)
    b.load_bin(f.getvalue())
    mel = synth_mel(24, 7) / sp.max_abs_value
    for m in (a, b):
        m.set_seed(11)
        m.generate(mel[None], True, 1000, 100, hp.mu_law, sp.preemphasize,
                   progress_callback=lambda *x: None)
    assert np.array_equal(a.last_labels, b.last_labels)


@pytest.mark.parametrize('mt,bits', [('fatchord-wavernn', 9), ('geneing-wavernn', 10)])
def test_fp16_bin_model_equals_fp16_rounded_state_dict(mt, bits):
    """An elSize-2 file runs as the state dict rounded to fp16 (the reader widens exactly)."""
    from wavernn_amd import convert
    from wavernn_amd.base import hparams_for
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    hp = hparams_for(mt).copy(bits=bits)
    sd = pruned_state_dict(hp, mt, keep=0.5)
    sd16 = {k: (v.astype(np.float16).astype(np.float32) if v.dtype == np.float32 else v)
            for k, v in sd.items()}
    f = io.BytesIO()
    convert.write_bin(f, sd, hp, mt, el_size=2)
    a, b = _model(hp, mt), _model(hp, mt)
    a.load_state_dict(sd16)
    b.load_bin(f.getvalue())
    mel = synth_mel(24, 7) / sp.max_abs_value
    for m in (a, b):
        m.set_seed(11)
        m.generate(mel[None], True, 1000, 100, hp.mu_law, sp.preemphasize,
                   progress_callback=lambda *x: None)
    assert np.array_equal(a.last_labels, b.last_labels)


def test_libwavernn_vocoder_chunks_match_oracle(tmp_path):
    import torch
    from oracle.wavernn_oracle import oracle_infer_waveform
    from wavernn_amd import convert
    from wavernn_amd.base import hparams_for
    from wavernn_amd.hparams import sp
    from wavernn_amd.libwavernn import Vocoder
    from wavernn_amd.synth import synth_mel
    mt = 'runtimeracer-wavernn'
    hp = hparams_for(mt)
    sd = pruned_state_dict(hp, mt, seed=5, keep=0.6)
    path = tmp_path / 'voc.bin'
    with open(path, 'wb') as f:
        convert.write_bin(f, sd, hp, mt)
    v = Vocoder(str(path), mt, verbose=False)
    v.setRandomSeed(21)
    v.load(max_threads=3)
    mel = synth_mel(60, 9)
    wav = v.vocode_mel(mel.copy())
    assert wav.shape == (60 * sp.hop_size,) and np.isfinite(wav).all()
    # the chunks of that call, re-run on the device and on the oracle
    hp_w = hparams_for(mt)
    wave_len = mel.shape[1] * sp.hop_size
    tgt = max(hp_w.gen_target, int(np.ceil((wave_len - hp_w.gen_overlap) / 3 - hp_w.gen_overlap)))
    chunks = v.fold_mel_with_overlap(mel / sp.max_abs_value, tgt, hp_w.gen_overlap)
    assert len(chunks) >= 2
    m = v._model
    m.set_seed(21)
    dev = [torch.from_numpy(np.ascontiguousarray(c, np.float32)).cuda() for c in chunks]
    lab, roff, S = m.generate_batch_device(dev, False, 0, 0)
    lab = lab.cpu().numpy()
    for u, c in enumerate(chunks):
        ref = oracle_infer_waveform(sd, hp, mt, c * sp.max_abs_value, batched=False, seed=21,
                                    stream=u)
        assert np.array_equal(lab[roff[u]:roff[u + 1]], ref['labels']), f'chunk {u}'
