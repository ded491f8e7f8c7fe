"""GPU side of tools/near_tie.py: for a parity-sweep case whose labels differ from the oracle,
record the kernels' logits (teacher-forced: the labels agree up to that step) at the first
differing (row, step) and compare them with the oracle's: the logit error against the decision's
top-1 / top-2 gap. Usage (GPU box):
  python tools/near_tie_gpu.py <default|peaked> <weight_seed> <noise_seed> <utts> <utterance> <row> <step> [fatchord|runtimeracer]
(mel seed of utterance u = 200 + case + 1000 u as in tools/parity_sweep.py; pass the sweep's
mel_seed of utterance 0 minus 200 as the case through weight_seed - 100)."""
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
from wavernn_amd.model import WaveRNN
from wavernn_amd.synth import synth_mel, synth_state_dict

kind, wseed, nseed, utts, u, row, step = sys.argv[1], *map(int, sys.argv[2:8])
topo = sys.argv[8] if len(sys.argv) > 8 else 'fatchord'
MT = topo + '-wavernn'
BITS, TARGET, OVERLAP = (10, 6000, 1000) if topo == 'runtimeracer' else (9, 11000, 550)
case = wseed - 100
stats = dict(gru_scale=3.0, fc_scale=2.0, logit_scale=16.0) if kind == 'peaked' else {}
torch.set_num_threads(16)
hp = hparams_for(MT).copy(bits=BITS, mode='RAW')
sd = synth_state_dict(hp, MT, seed=wseed, **stats)
m = WaveRNN(hp.rnn_dims, hp.fc_dims, hp.bits, hp.pad, hp.upsample_factors, sp.num_mels,
            hp.compute_dims, hp.res_out_dims, hp.res_blocks, sp.hop_size, sp.sample_rate,
            mode='RAW', model_type=MT, device=0)
m.load_state_dict(sd)
m.set_seed(nseed)
mels = [synth_mel(1000, 200 + case + 1000 * k) for k in range(utts)]
devs = [torch.from_numpy((x / sp.max_abs_value).astype(np.float32)).cuda() for x in mels]
m.set_debug_steps([step])
out, roff, S = m.generate_batch_device(devs, True, TARGET, OVERLAP)
lab = out.cpu().numpy()[roff[u]:roff[u + 1]]
g_log = m.debug_logits(step, [roff[u] + row])[0].astype(np.float64)
sdt = {k: torch.from_numpy(np.asarray(v)) if not torch.is_tensor(v) else v for k, v in sd.items()}
o = OracleWaveRNN(sdt, hp, MT).generate(
    torch.from_numpy((mels[u] / sp.max_abs_value)[None].astype(np.float32)), True, TARGET, OVERLAP,
    hp.mu_law, True, seed=nseed, stream=u, max_steps=step + 1, record_logits=[step], post=False)
o_log = o['logits'][step][row].astype(np.float64)
q = philox.raw_exp_noise(nseed, u, [step], np.arange(lab.shape[0]), 2 ** hp.bits)[0][row]


def decide(lg):
    p = F.softmax(torch.from_numpy(lg.astype(np.float32))[None], dim=1)[0]
    r = (p / p.sum()) / torch.from_numpy(q)
    t = torch.topk(r, 2)
    return [int(i) for i in t.indices], float(np.log(float(t.values[0])) - np.log(float(t.values[1])))


(gk, ggap), (ok, ogap) = decide(g_log), decide(o_log)
print(json.dumps({'model': MT, 'kind': kind, 'case': case, 'utts': utts, 'utterance': u, 'row': row, 'step': step,
                  'labels_equal_before_step': bool(np.array_equal(lab[:, :step], o['labels'][:, :step])),
                  'gpu_label': int(lab[row, step]), 'oracle_label': int(o['labels'][row, step]),
                  'oracle_top2': ok, 'oracle_gap': ogap, 'gpu_top2': gk, 'gpu_gap': ggap,
                  'max_abs_dlogit_row': float(np.max(np.abs(g_log - o_log))),
                  'dlogit_top2': [float(g_log[ok[0]] - o_log[ok[0]]), float(g_log[ok[1]] - o_log[ok[1]])],
                  'max_abs_logit': float(np.max(np.abs(o_log)))}))
