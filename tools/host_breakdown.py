"""Host-side breakdown of one C2 bench step (generate_batch_device / D2H / post-processing),
wall clock with device syncs, on the GPU box. Usage: python tools/host_breakdown.py [--timing]"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'real-time-voice-cloning_amd'), REPO]
import numpy as np
import torch
from wavernn_amd.model import WaveRNN
from wavernn_amd.hparams import wavernn_fatchord, sp
from wavernn_amd.synth import synth_state_dict, synth_mel

hp = wavernn_fatchord.copy(bits=9, mode='RAW')
sd = synth_state_dict(hp, 'fatchord-wavernn', seed=0)
m = WaveRNN(hp.rnn_dims, hp.fc_dims, hp.bits, hp.pad, hp.upsample_factors, sp.num_mels,
            hp.compute_dims, hp.res_out_dims, hp.res_blocks, sp.hop_size, sp.sample_rate,
            mode='RAW', model_type='fatchord-wavernn', device=0)
m.load_state_dict(sd)
m.set_seed(1234)
if '--timing' in sys.argv:
    m.enable_stage_timing(True)
mel = torch.from_numpy((synth_mel(1000, seed=0) / sp.max_abs_value).astype(np.float32)).cuda()
T = {}
for it in range(6):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out, roff, S = m.generate_batch_device([mel], True, 11000, 550)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    host = out.cpu().numpy()
    t3 = time.perf_counter()
    wav = m.postprocess_rows(host, 1000, True, 11000, 550, hp.mu_law, sp.preemphasize)
    t4 = time.perf_counter()
    if it >= 2:
        for k, v in (('call', t1 - t0), ('sync', t2 - t1), ('d2h', t3 - t2), ('post', t4 - t3),
                     ('total', t4 - t0)):
            T.setdefault(k, []).append(v * 1e3)
print({k: round(float(np.median(v)), 3) for k, v in T.items()}, 'ms (median of 4)')
