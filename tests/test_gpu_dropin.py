"""Drop-in round trip on the GPU: checkpoint file -> vocoder.inference.load_model -> set_seed ->
infer_waveform, exactly as demo_cli.py / the toolbox call it (vocoder/inference.py:11-101).

The checkpoint is the training format ``{"model_state": state_dict, "model_type": ...}``
(vocoder/train.py:308-324) written with torch.save from the seeded synthetic weights of a
golden case whose hparams are the file defaults (fatchord / runtimeracer 10-bit RAW, default
gen_target / gen_overlap), so ``load_model`` builds the model from the module hparams with no
override -- the reference's own path -- and the result must equal the waveform the real
reference infer_waveform produced for that case (tests/golden/gen_golden.py).
"""
import numpy as np
import pytest

from conftest import golden_case, hparams_of

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('name', ['fatchord_raw10_defaults', 'runtimeracer_raw10_defaults'])
def test_checkpoint_load_infer_waveform_equals_reference(name, tmp_path):
    import torch
    from vocoder import inference as vinf  # the drop-in module name of the reference
    from wavernn_amd.base import hparams_for
    from wavernn_amd.synth import synth_state_dict, synth_mel
    meta, gold = golden_case(name)
    hp = hparams_of(meta)
    d = hparams_for(meta['model_type'])
    assert (hp.bits, hp.mode) == (d.bits, d.mode), 'case must use the file-default hparams'
    sd = synth_state_dict(hp, meta['model_type'], seed=meta['weight_seed'],
                          logit_scale=meta['logit_scale'])
    ckpt = tmp_path / 'vocoder.pt'
    torch.save({'model_state': {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()},
                'model_type': meta['model_type'], 'step': 1234}, str(ckpt))
    vinf.load_model(str(ckpt), verbose=False)
    assert vinf.is_loaded()
    vinf.set_seed(meta['noise_seed'])
    calls = []
    wav = vinf.infer_waveform(synth_mel(meta['n_frames'], meta['mel_seed']),
                              progress_callback=lambda *c: calls.append(c[0]))
    assert calls == list(range(0, meta['seq_len'], 100))
    assert wav.dtype == np.float64 and wav.shape == gold['wav'].shape
    assert np.array_equal(wav, gold['wav'])
