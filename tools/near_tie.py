"""Is a label difference of the parity sweep a near-tie of the reference's own decision?
For one tools/parity_sweep.py case (weights / mel / noise seeds, noise stream) and the (row,
step) of the first difference, on the host: (1) the oracle's top-1 / top-2 gap there (log of the
fp32 probs / q ratios, the margin a summation-order change must overcome), and (2) the first
difference of that row between the oracle and the oracle with every Linear in float64 rounded to
fp32 (tests/golden/gen_golden.py perturbed_first_div: another valid fp32 evaluation of the same
model). CPU only. Usage:
  python tools/near_tie.py <default|peaked> <weight_seed> <mel_seed> <noise_seed> <stream> <row> <step>
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'real-time-voice-cloning_amd'), REPO]
import numpy as np
import torch
import torch.nn.functional as F

from oracle import philox
from oracle.wavernn_oracle import OracleWaveRNN
from wavernn_amd.base import hparams_for
from wavernn_amd.hparams import sp
from wavernn_amd.synth import synth_mel, synth_state_dict

kind, wseed, mseed, nseed, stream, row, step = sys.argv[1], *map(int, sys.argv[2:8])
stats = dict(gru_scale=3.0, fc_scale=2.0, logit_scale=16.0) if kind == 'peaked' else {}
torch.set_num_threads(int(os.environ.get('THREADS', '8')))
hp = hparams_for('fatchord-wavernn').copy(bits=9, mode='RAW')
sd = {k: torch.from_numpy(np.asarray(v)) if not torch.is_tensor(v) else v
      for k, v in synth_state_dict(hp, 'fatchord-wavernn', seed=wseed, **stats).items()}
mel = synth_mel(1000, mseed)
mel_t = torch.from_numpy((mel / sp.max_abs_value)[None, ...].astype(np.float32))
res = {}
for name in ('fp32', 'f64_linear'):
    m = OracleWaveRNN(sd, hp, 'fatchord-wavernn')
    if name == 'f64_linear':
        m._lin = lambda n, x, m=m: F.linear(x.double(), m.sd[n + '.weight'].double(),
                                            m.sd[n + '.bias'].double()).float()
    o = m.generate(mel_t, True, 11000, 550, hp.mu_law, True, seed=nseed, stream=stream,
                   max_steps=step + 1, record_logits=[step], post=False)
    res[name] = o
lg = torch.from_numpy(res['fp32']['logits'][step])
q = torch.from_numpy(philox.raw_exp_noise(nseed, stream, [step], np.arange(lg.shape[0]), 2 ** hp.bits)[0])
post = F.softmax(lg, dim=1)
ratio = (post / post.sum(-1, keepdim=True)) / q
top = torch.topk(ratio[row], 2)
gap = float(np.log(top.values[0].double()) - np.log(top.values[1].double()))
d = np.nonzero(res['fp32']['labels'][row] != res['f64_linear']['labels'][row])[0]
print(json.dumps({'kind': kind, 'weight_seed': wseed, 'mel_seed': mseed, 'noise_seed': nseed,
                  'stream': stream, 'row': row, 'step': step,
                  'oracle_top2_gap': gap, 'top2_classes': [int(i) for i in top.indices],
                  'max_abs_logit': float(lg[row].abs().max()),
                  'f64_linear_first_div_in_row': int(d[0]) if len(d) else None}))
