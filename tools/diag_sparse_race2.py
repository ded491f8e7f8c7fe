"""Diagnostic: test_gpu_sparse.py's order in one process, three times over: each pruned fixture
on the sparse path, then sparse vs dense with the logit capture, every captured (step, row)
against the reference's logits. Prints the entries whose error exceeds 1e-7."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'tests'), os.path.join(REPO, 'real-time-voice-cloning_amd'), REPO]


def main(rounds='3'):
    from conftest import golden_case, golden_meta
    from test_gpu_parity import make_model
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    pruned = sorted(k for k, v in golden_meta().items() if v.get('prune'))
    fat = [k for k in pruned if golden_meta()[k]['model_type'] == 'fatchord-wavernn']

    def run(name, sparse, dbg):
        meta, gold = golden_case(name)
        os.environ['WRNN_SPARSE'] = '1' if sparse else '0'
        m, hp, sd = make_model(meta)
        m.set_engine('persist')
        steps = [int(s) for s in gold['logits_steps']][:4]
        if dbg:
            m.set_debug_steps(steps)
        mel = synth_mel(meta['n_frames'], meta['mel_seed']) / sp.max_abs_value
        m.generate(mel[None], meta['batched'], meta['target'], meta['overlap'], hp.mu_law,
                   sp.preemphasize, progress_callback=lambda *a: None)
        out = None
        if dbg:
            rows = range(meta['num_folds'])
            lg = np.stack([m.debug_logits(s, rows) for s in steps]).astype(np.float64)
            ref = gold['logits'][:len(steps)]
            err = np.abs(lg - ref).max(axis=2)
            out = [(steps[i], r, float(err[i, r])) for i, r in np.argwhere(err > 1e-7)]
        lab_ok = None if meta['mode'] == 'MOL' else bool(np.array_equal(m.last_labels, gold['labels']))
        return out, lab_ok, m.plan_info(), m.sparse_info()['last_call']

    for rd in range(int(rounds)):
        for name in pruned:
            _, ok, plan, sp_ = run(name, True, False)
            print(f'round {rd} {name} sparse plain: labels==gold {ok} plan {plan} sparse {sp_}', flush=True)
        for name in fat:
            for sparse in (True, False):
                bad, ok, plan, sp_ = run(name, sparse, True)
                print(f'round {rd} {name} sparse={sparse} dbg: labels==gold {ok} plan {plan} ran sparse {sp_}; '
                      f'captures off the reference by > 1e-7: {bad[:8]}', flush=True)


if __name__ == '__main__':
    main(*sys.argv[1:])
