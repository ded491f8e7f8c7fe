"""End-to-end callers of the vocoder against the reference, CPU.

Fixtures: tests/golden/gen_e2e_golden.py ran the reference's own SpeakerEncoder, Tacotron and
text front end on the same seeded weights / inputs (Tacotron prenet dropout from the shared
``DropoutStream``). The PyTorch CPU kernels are the same, so equality is exact.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

G = np.load(os.path.join(GOLDEN, 'e2e_models.npz'))
TACO_SEED, ENC_SEED, DROP_SEED, STEPS = (int(v) for v in G['seeds'])


def tacotron(device='cpu'):
    from synthesizer.inference import build_tacotron
    from synthesizer.tacotron import synth_tacotron_state_dict
    m = build_tacotron(device)
    sd = synth_tacotron_state_dict(m, TACO_SEED)
    sd['decoder.stop_proj.bias'] = torch.full_like(sd['decoder.stop_proj.bias'], -8.0)
    m.load_state_dict(sd)
    return m.eval()


def run_tacotron(device='cpu'):
    from synthesizer import tacotron as T
    m = tacotron(device)
    T.set_dropout_stream(DROP_SEED)
    try:
        mel, lin, attn = m.generate(torch.from_numpy(G['chars']).to(device),
                                    torch.from_numpy(G['spk']).to(device), steps=STEPS)
        calls = T._dropout.calls
    finally:
        T.set_dropout_stream(None)
    return mel.cpu().numpy(), lin.cpu().numpy(), attn.cpu().numpy(), calls


def test_tacotron_generate_matches_reference():
    torch.set_num_threads(8)
    mel, lin, attn, calls = run_tacotron()
    assert calls == int(G['dropout_calls'][0])
    assert mel.shape == G['mel_out'].shape and lin.shape == G['linear'].shape
    np.testing.assert_array_equal(mel, G['mel_out'])
    np.testing.assert_array_equal(lin, G['linear'])
    np.testing.assert_array_equal(attn, G['attn'])


def test_speaker_encoder_matches_reference():
    from encoder.model import SpeakerEncoder, synth_encoder_state_dict
    m = SpeakerEncoder('cpu')
    m.load_state_dict(synth_encoder_state_dict(m, ENC_SEED))
    m.eval()
    frames = np.random.default_rng(int(G['enc_frames_seed'][0])).uniform(0, 2, (3, 160, 40)).astype(np.float32)
    with torch.no_grad():
        e = m(torch.from_numpy(frames)).numpy()
    np.testing.assert_array_equal(e, G['enc_embeds'])


def test_text_to_sequence_matches_reference():
    from synthesizer.text import sequence_to_text, text_to_sequence
    ref = json.load(open(os.path.join(GOLDEN, 'e2e_text.json')))
    for text, seq in ref.items():
        assert text_to_sequence(text.strip(), ['english_cleaners']) == seq, text
        assert sequence_to_text(seq).endswith('~')


def test_partial_slices_and_mel_features():
    from encoder import inference as enc
    from encoder.audio import mel_filterbank, wav_to_mel_spectrogram
    w, m = enc.compute_partial_slices(16000 * 3)
    assert [s.start for s in m][:3] == [0, 80, 160] and all(s.stop - s.start == 160 for s in m)
    assert all(ws.stop - ws.start == 160 * 160 for ws in w)
    fb = mel_filterbank(16000, 400, 40)
    assert fb.shape == (40, 201) and (fb >= 0).all()
    # a 1 kHz tone puts its energy in the filters around 1 kHz (Slaney mel)
    t = np.arange(16000) / 16000.0
    frames = wav_to_mel_spectrogram(np.sin(2 * np.pi * 1000 * t).astype(np.float32))
    assert frames.shape == (101, 40) and frames.dtype == np.float32
    peak = int(np.argmax(frames[50]))
    centres = (np.argmax(fb, axis=1) * 40.0)
    assert abs(centres[peak] - 1000) < 150
