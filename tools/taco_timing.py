"""Diagnostic: Tacotron generate on the GPU, eager loop vs HIP-graph loop (B utterances,
400 decoder steps, random weights, stop disabled)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'real-time-voice-cloning_amd'))
import numpy as np
import torch

from synthesizer.inference import build_tacotron
from synthesizer.tacotron import set_dropout_stream, synth_tacotron_state_dict

B = int(os.environ.get('B', '8'))
m = build_tacotron('cpu')
sd = synth_tacotron_state_dict(m, 1)
sd['decoder.stop_proj.bias'] = torch.full_like(sd['decoder.stop_proj.bias'], -8.0)
m.load_state_dict(sd)
m = m.cuda().eval()
rng = np.random.default_rng(0)
chars = torch.from_numpy(rng.integers(1, 60, (B, 70))).cuda()
spk = torch.from_numpy(rng.normal(size=(B, 768)).astype(np.float32)).cuda()
for seed in (None, 3):
    set_dropout_stream(seed)
    for graph in (False, True, True):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mel, lin, att = m.generate(chars, spk, steps=400, graph=graph)
        torch.cuda.synchronize()
        print(f'stream={seed} graph={graph}: {time.perf_counter() - t0:.3f} s, frames {mel.shape[2]}',
              flush=True)
