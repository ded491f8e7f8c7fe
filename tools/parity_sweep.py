"""Full-size C2 parity sweep on the GPU box: several (weights, mel, noise) seeds, the HIP path
(generate_batch_device, the bench's path) against the oracle on the host, labels and f64
waveform compared. One JSON line per case.
Usage: python tools/parity_sweep.py [n_cases] [default|peaked] [utts] [fatchord|runtimeracer]
  peaked: the trained-like statistics of tests/golden fatchord_raw9_c2_peaked (GRU weights x3,
          hidden fc x2, output layer x16: |logit| up to ~20, peaked posteriors)
  utts:   utterances per call (8 = the C4 per-GPU shape: wide + register-resident launches);
          every utterance is checked on its own noise stream
  runtimeracer: the fork's default topology at its defaults (10 bits, target 6000 / overlap
          1000); 8 utterances run on the runtimeracer wide kernel"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'real-time-voice-cloning_amd'), REPO]
import numpy as np
import torch

from oracle.wavernn_oracle import oracle_infer_waveform
from wavernn_amd.base import hparams_for
from wavernn_amd.hparams import sp
from wavernn_amd.model import WaveRNN
from wavernn_amd.synth import synth_mel, synth_state_dict

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
kind = sys.argv[2] if len(sys.argv) > 2 else 'default'
utts = int(sys.argv[3]) if len(sys.argv) > 3 else 1
topo = sys.argv[4] if len(sys.argv) > 4 else 'fatchord'
MT = topo + '-wavernn'
BITS, TARGET, OVERLAP = (10, 6000, 1000) if topo == 'runtimeracer' else (9, 11000, 550)
FRAMES = 1000
stats = dict(gru_scale=3.0, fc_scale=2.0, logit_scale=16.0) if kind == 'peaked' else {}
torch.set_num_threads(16)
for case in range(n):
    wseed, mseed, nseed = 100 + case, 200 + case, 300 + case
    hp = hparams_for(MT).copy(bits=BITS, mode='RAW')
    sd = synth_state_dict(hp, MT, seed=wseed, **stats)
    m = WaveRNN(hp.rnn_dims, hp.fc_dims, hp.bits, hp.pad, hp.upsample_factors, sp.num_mels,
                hp.compute_dims, hp.res_out_dims, hp.res_blocks, sp.hop_size, sp.sample_rate,
                mode='RAW', model_type=MT, device=0)
    m.load_state_dict(sd)
    m.set_seed(nseed)
    mels = [synth_mel(FRAMES, mseed + 1000 * u) for u in range(utts)]
    devs = [torch.from_numpy((mel / sp.max_abs_value).astype(np.float32)).cuda() for mel in mels]
    out, roff, S = m.generate_batch_device(devs, True, TARGET, OVERLAP)
    lab_all = out.cpu().numpy()
    engine = m.last_engine()
    # the last utterance (every launch kind of the plan holds some of its rows at utts = 8 ...)
    # and the first
    for u in sorted({0, utts - 1}):
        lab = lab_all[roff[u]:roff[u + 1]]
        wav = m.postprocess_rows(lab, FRAMES, True, TARGET, OVERLAP, hp.mu_law, sp.preemphasize)
        t0 = time.time()
        ref = oracle_infer_waveform(sd, hp, MT, mels[u], target=TARGET, overlap=OVERLAP,
                                    seed=nseed, stream=u)
        d = np.argwhere(lab != ref['labels'])
        print(json.dumps({'case': case, 'model': MT, 'kind': kind, 'utts': utts, 'utterance': u, 'weight_seed': wseed,
                          'mel_seed': mseed + 1000 * u, 'noise_seed': nseed,
                          'rows': int(lab.shape[0]), 'steps': int(lab.shape[1]),
                          'engine': engine, 'labels_equal': bool(len(d) == 0),
                          'mismatches': int(len(d)),
                          'first_divergence': None if len(d) == 0 else [int(v) for v in d[np.argmin(d[:, 1])]],
                          'wave_bit_exact': bool(np.array_equal(wav, ref['wav'])),
                          'oracle_s': round(time.time() - t0, 1)}), flush=True)
