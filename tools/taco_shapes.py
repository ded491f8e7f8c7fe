"""Diagnostic: first-call cost of new (batch, text length) shapes in the Tacotron on the GPU."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'real-time-voice-cloning_amd'))
import numpy as np
import torch

from synthesizer.inference import build_tacotron
from synthesizer.tacotron import set_dropout_stream, synth_tacotron_state_dict

m = build_tacotron('cpu')
sd = synth_tacotron_state_dict(m, 1)
sd['decoder.stop_proj.bias'] = torch.full_like(sd['decoder.stop_proj.bias'], -8.0)
m.load_state_dict(sd)
m = m.cuda().eval()
set_dropout_stream(3)
rng = np.random.default_rng(0)
for B, T, steps in [(1, 9, 20), (8, 70, 100), (8, 70, 100), (8, 71, 100), (7, 64, 100), (8, 70, 400)]:
    chars = torch.from_numpy(rng.integers(1, 60, (B, T))).cuda()
    spk = torch.from_numpy(rng.normal(size=(B, 768)).astype(np.float32)).cuda()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    enc = m.encoder(chars, spk)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    mel, lin, att = m.generate(chars, spk, steps=steps)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f'B={B} T={T} steps={steps}: encoder {t1 - t0:.3f} s, generate {t2 - t1:.3f} s', flush=True)
