"""Golden fixtures of the end-to-end path's callers (survey container only).

Imports the reference's speaker encoder (``encoder/model.py``), Tacotron
(``synthesizer/models/tacotron.py``) and text front end (``synthesizer/utils/text.py``) from
/root/reference with import shims for packages absent from this image (``unidecode`` as the
identity -- only ASCII text is recorded --, ``inflect`` / ``phonemizer`` as unused stubs, plus the
vocoder shims of gen_golden.py), loads seeded stand-in weights built by this repository's own
``synth_*_state_dict`` helpers (loading them into the reference modules strictly also proves the
state-dict names match), and records:

* ``SpeakerEncoder.forward`` on seeded mel frames (3 x 160 x 40);
* ``Tacotron.generate`` on two seeded-embedding utterances, with the prenet dropout
  (``F.dropout(..., training=True)``, tacotron.py:150-157) drawn from
  ``synthesizer.tacotron.DropoutStream`` -- the reference is patched to call the same stream;
* ``text_to_sequence`` of a few ASCII sentences without digits (english_cleaners).

Usage:  python tests/golden/gen_e2e_golden.py
"""
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden  # noqa: E402  (paths, vocoder shims)

import torch  # noqa: E402

from encoder.model import SpeakerEncoder as OurEncoder, synth_encoder_state_dict  # noqa: E402
from synthesizer.inference import build_tacotron  # noqa: E402
from synthesizer.tacotron import DropoutStream, synth_tacotron_state_dict  # noqa: E402

TEXTS = ["Hello world.", "The quick brown fox jumps over the lazy dog!",
         "Dr. Smith met Mr. Jones on Jan. fourth, near St. Paul's.",
         "  Multiple   spaces,  (parentheses) and \"quotes\"; semi: colons? yes - no. "]
TACO_SEED, ENC_SEED, DROP_SEED, STEPS = 7, 8, 9, 60


def install_e2e_shims():
    gen_golden.install_shims()
    uni = types.ModuleType('unidecode')
    uni.unidecode = lambda s: s
    sys.modules['unidecode'] = uni
    inf = types.ModuleType('inflect')
    inf.engine = lambda: None
    sys.modules['inflect'] = inf
    ph = types.ModuleType('phonemizer')
    php = types.ModuleType('phonemizer.phonemize')
    php.phonemize = lambda *a, **k: ''
    sys.modules['phonemizer'] = ph
    sys.modules['phonemizer.phonemize'] = php
    for m in [m for m in list(sys.modules) if m == 'encoder' or m.startswith('encoder.') or
              m == 'synthesizer' or m.startswith('synthesizer.')]:
        del sys.modules[m]


def main():
    torch.set_num_threads(8)
    # our modules first (state-dict templates), then the reference ones
    our_taco = build_tacotron('cpu')
    taco_sd = synth_tacotron_state_dict(our_taco, TACO_SEED)
    # stop tokens well below 0.5 so the decoder runs all STEPS iterations (random weights
    # would otherwise stop at the first allowed step)
    taco_sd['decoder.stop_proj.bias'] = torch.full_like(taco_sd['decoder.stop_proj.bias'], -8.0)
    our_enc = OurEncoder('cpu')
    enc_sd = synth_encoder_state_dict(our_enc, ENC_SEED)
    install_e2e_shims()
    from config.hparams import sp, sv2tts, tacotron as hpt
    from encoder.model import SpeakerEncoder
    from synthesizer.models.tacotron import Tacotron
    from synthesizer.utils.symbols import symbols
    from synthesizer.utils.text import text_to_sequence

    # --- speaker encoder
    enc = SpeakerEncoder(torch.device('cpu'))
    enc.load_state_dict(enc_sd)
    enc.eval()
    frames = np.random.default_rng(3).uniform(0, 2, (3, 160, 40)).astype(np.float32)
    with torch.no_grad():
        embeds = enc(torch.from_numpy(frames)).numpy()

    # --- Tacotron
    taco = Tacotron(embed_dims=hpt.embed_dims, num_chars=len(symbols), encoder_dims=hpt.encoder_dims,
                    decoder_dims=hpt.decoder_dims, n_mels=sp.num_mels, fft_bins=sp.num_mels,
                    postnet_dims=hpt.postnet_dims, encoder_K=hpt.encoder_K, lstm_dims=hpt.lstm_dims,
                    postnet_K=hpt.postnet_K, num_highways=hpt.num_highways, dropout=hpt.dropout,
                    stop_threshold=hpt.stop_threshold,
                    speaker_embedding_size=sv2tts.speaker_embedding_size)
    taco.load_state_dict(taco_sd)
    taco.eval()
    seqs = [text_to_sequence(t.strip(), ['english_cleaners']) for t in TEXTS]
    chars = np.zeros((2, max(len(seqs[0]), len(seqs[1]))), np.int64)
    for i in range(2):
        chars[i, :len(seqs[i])] = seqs[i]
    spk = np.random.default_rng(4).normal(size=(2, sv2tts.speaker_embedding_size)).astype(np.float32)
    spk /= np.linalg.norm(spk, axis=1, keepdims=True)
    stream = DropoutStream(DROP_SEED)
    real = torch.nn.functional.dropout
    torch.nn.functional.dropout = lambda x, p=0.5, training=True, inplace=False: stream(x, p)
    try:
        with torch.no_grad():
            mel_out, linear, attn = taco.generate(torch.from_numpy(chars), torch.from_numpy(spk),
                                                  steps=STEPS)
    finally:
        torch.nn.functional.dropout = real
    np.savez_compressed(os.path.join(HERE, 'e2e_models.npz'), enc_frames_seed=np.array([3]),
                        enc_embeds=embeds, chars=chars, spk=spk, mel_out=mel_out.numpy(),
                        linear=linear.numpy(), attn=attn.numpy(),
                        seeds=np.array([TACO_SEED, ENC_SEED, DROP_SEED, STEPS]),
                        dropout_calls=np.array([stream.calls]))
    with open(os.path.join(HERE, 'e2e_text.json'), 'w') as f:
        json.dump({t: s for t, s in zip(TEXTS, seqs)}, f, indent=1)
    print('encoder', embeds.shape, 'tacotron', tuple(linear.shape), 'dropout calls', stream.calls)


if __name__ == '__main__':
    main()
