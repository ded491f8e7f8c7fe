"""Full-size parity sweep as a gate (VERDICT r4 "Next" 1): several (weights, mel, noise) seed
triples per headline shape, the bench's path (generate_batch_device) against the oracle run on
the host with the same seed and stream, labels compared per utterance.

A label difference is allowed only as a NEAR-TIE (tests/near_tie_util.py), decided at each
diverged row's first differing step: the call is re-run with the kernels' logits recorded there
(teacher-forced: the row's labels agree before it), the oracle is re-run up to it, and
  * the kernel's label there must be the exact decision on the kernel's OWN logits
    (wrnn_debug_decide, csrc/cand_key.h) -- the kernels implement the decision exactly;
  * the oracle's margin between its label and the kernel's, v_o(k_o) - v_o(k_g) with v = l + G
    formed exactly, must not exceed 2 x the kernel's logit error on those two classes plus the
    reference's own fp32 rounding of the decision (tests/test_decision.py eps_ref).
Anything else fails: a flip that is not explained by summation-order logit error at a tie.
Shapes (BASELINE.json configs[1] and the runtimeracer fork's default topology at the C4 shape):
  c2    fatchord RAW 9-bit, one 1000-frame mel, target 11000 / overlap 550 (18 x 12,100)
  c2pk  the same with trained-like statistics (tests/golden fatchord_raw9_c2_peaked's knobs)
  rr8   runtimeracer RAW 10-bit, 8 x 1000-frame mels, 6000 / 1000 (232 rows, wide launches);
        utterances 0 and 7 checked
  rr8pk the same with the trained-like statistics; rr8pk-reg on the register-resident kernel
        (these two with WRNN_SWEEP_ALL=1)
Seeds as tools/parity_sweep.py (weights 100 + case, mel 200 + case + 1000 u, noise 300 + case),
so the round-4 sweep's recorded flips (profiles/r04/parity_sweep/) are among the cases. With
WRNN_SWEEP_OUT set, one JSON line per utterance is appended there (DESIGN.md §5 numbers).
Reference: vocoder/models/fatchord_version.py:192-236, runtimeracer_version.py:244-281.
"""
import json
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHAPES = {
    'c2': dict(topo='fatchord', bits=9, target=11000, overlap=550, utts=1, stats={}),
    'c2pk': dict(topo='fatchord', bits=9, target=11000, overlap=550, utts=1,
                 stats=dict(gru_scale=3.0, fc_scale=2.0, logit_scale=16.0)),
    'rr8': dict(topo='runtimeracer', bits=10, target=6000, overlap=1000, utts=8, stats={}),
    'rr8pk': dict(topo='runtimeracer', bits=10, target=6000, overlap=1000, utts=8,
                  stats=dict(gru_scale=3.0, fc_scale=2.0, logit_scale=16.0)),
    # the same on the register-resident runtimeracer kernel (8 launches of <= 4 rows per group),
    # its flip count next to the wide kernel's on the same seeds
    'rr8pk-reg': dict(topo='runtimeracer', bits=10, target=6000, overlap=1000, utts=8,
                      stats=dict(gru_scale=3.0, fc_scale=2.0, logit_scale=16.0), wide='0'),
}
# the gate (>= 4 seed triples x {C2 default, C2 trained-like, runtimeracer 8
# utterances}); WRNN_SWEEP_ALL=1 adds the trained-like runtimeracer cases on both kernels (the
# DESIGN.md §5 table; ~95 s more)
_ALL = os.environ.get('WRNN_SWEEP_ALL') == '1'
CASES = [(shape, case) for shape in SHAPES for case in range(2 if shape.startswith('rr8pk') else 4)
         if _ALL or not shape.startswith('rr8pk')]


def _build(shape, case):
    import torch
    from wavernn_amd.base import hparams_for
    from wavernn_amd.hparams import sp
    from wavernn_amd.model import WaveRNN
    from wavernn_amd.synth import synth_mel, synth_state_dict
    c = SHAPES[shape]
    mt = c['topo'] + '-wavernn'
    hp = hparams_for(mt).copy(bits=c['bits'], mode='RAW')
    sd = synth_state_dict(hp, mt, seed=100 + case, **c['stats'])
    m = WaveRNN(hp.rnn_dims, hp.fc_dims, hp.bits, hp.pad, hp.upsample_factors, sp.num_mels, hp.compute_dims,
                hp.res_out_dims, hp.res_blocks, sp.hop_size, sp.sample_rate, mode='RAW', model_type=mt, device=0)
    m.load_state_dict(sd)
    mels = [synth_mel(1000, 200 + case + 1000 * u) for u in range(c['utts'])]
    dev = [torch.from_numpy((x / sp.max_abs_value).astype(np.float32)).cuda() for x in mels]
    return m, hp, sd, mt, mels, dev


def _run(m, dev, c, nseed, steps=None):
    """The call; with `steps`, the logits recorded there: {step: (all rows, n_classes)}."""
    m.set_seed(nseed)
    m.set_debug_steps(steps)
    try:
        out, roff, S = m.generate_batch_device(dev, True, c['target'], c['overlap'])
        lab = out.cpu().numpy()
        logs = {s: m.debug_logits(s, range(lab.shape[0])) for s in (steps or [])}
        return lab, list(roff), logs
    finally:
        m.set_debug_steps(None)


@pytest.mark.parametrize('shape,case', CASES, ids=[f'{s}-{c}' for s, c in CASES])
def test_full_size_sweep_flips_only_at_near_ties(shape, case, monkeypatch):
    import torch
    from oracle.wavernn_oracle import OracleWaveRNN, oracle_infer_waveform
    from near_tie_util import analyse, divergence_steps, first_divergence_per_row
    from wavernn_amd import _abi
    from wavernn_amd.hparams import sp
    c = SHAPES[shape]
    nseed = 300 + case
    if 'wide' in c:
        monkeypatch.setenv('WRNN_PERSIST_WIDE', c['wide'])
    m, hp, sd, mt, mels, dev = _build(shape, case)
    lab_all, roff, _ = _run(m, dev, c, nseed)
    lib = _abi.load_library()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    out = os.environ.get('WRNN_SWEEP_OUT')
    bad = []
    for u in sorted({0, c['utts'] - 1}):
        lab = lab_all[roff[u]:roff[u + 1]]
        t0 = time.time()
        ref = oracle_infer_waveform(sd, hp, mt, mels[u], target=c['target'], overlap=c['overlap'],
                                    seed=nseed, stream=u, post=False)
        fd = first_divergence_per_row(lab, ref['labels'])
        rec = dict(shape=shape, case=case, utterance=u, rows=int(lab.shape[0]), steps=int(lab.shape[1]),
                   engine=m.last_engine(), plan=m.plan_info(), labels_equal=bool((fd < 0).all()),
                   rows_diverged=int((fd >= 0).sum()), mismatches=int((lab != ref['labels']).sum()),
                   oracle_s=round(time.time() - t0, 1))
        if (fd >= 0).any():
            steps = divergence_steps(fd)
            lab2, _, g_all = _run(m, dev, c, nseed, steps=steps)
            assert np.array_equal(lab2, lab_all), 'the re-run must reproduce the call'
            g = {s: v[roff[u]:roff[u + 1]] for s, v in g_all.items()}
            sdt = {k: torch.from_numpy(np.asarray(v)) if not torch.is_tensor(v) else v for k, v in sd.items()}
            o = OracleWaveRNN(sdt, hp, mt).generate(
                torch.from_numpy((mels[u] / sp.max_abs_value)[None].astype(np.float32)), True, c['target'],
                c['overlap'], hp.mu_law, True, seed=nseed, stream=u, max_steps=max(steps) + 1,
                record_logits=steps, post=False)
            _, recs = analyse(lib, nseed, u, lab, ref['labels'], g, o['logits'])
            rec['near_ties'] = recs
            bad += [r for r in recs if not r['near_tie']]
            if len(steps) < len({int(s) for s in fd if s >= 0}):
                rec['unanalysed_rows'] = int(sum(1 for s in fd if s > max(steps)))
        if out:
            with open(out, 'a') as f:
                f.write(json.dumps(rec) + '\n')
        print(json.dumps(rec))
    assert not bad, f'label differences that are not near-ties: {bad}'
