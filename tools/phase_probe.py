"""Diagnostic: one config-2 generate with per-phase stamps of one step (env WRNN_PHASE_STEP)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'real-time-voice-cloning_amd'))
import numpy as np
from wavernn_amd.model import WaveRNN
from wavernn_amd.hparams import sp, wavernn_fatchord
from wavernn_amd.synth import synth_state_dict, synth_mel
T = int(os.environ.get('FRAMES', '1000'))
hp = wavernn_fatchord.copy(bits=9, mode='RAW')
m = WaveRNN(hp.rnn_dims, hp.fc_dims, hp.bits, hp.pad, hp.upsample_factors, 80, hp.compute_dims,
            hp.res_out_dims, hp.res_blocks, 200, 16000, mode='RAW', model_type='fatchord-wavernn')
m.load_state_dict(synth_state_dict(hp, 'fatchord-wavernn', seed=0))
mel = synth_mel(T, 0) / 4.0
for i in range(2):
    t0 = time.time()
    m.generate(mel[None], True, 11000, 550, True, True, progress_callback=lambda *a: None)
    print('generate', time.time() - t0, m.timings, flush=True)
