"""Diagnostic: test_sparse_equals_dense_bit_for_bit's body verbatim (sparse handle, then dense
handle, both alive; captures read afterwards), N times on fatchord_raw10_pruned_defaults, after
the sparse-path runs of every pruned fixture. Reports every repetition whose sparse and dense
captures differ, with the (step, row) entries and their errors against the reference."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'tests'), os.path.join(REPO, 'real-time-voice-cloning_amd'), REPO]


def main(n='40', name='fatchord_raw10_pruned_defaults'):
    from conftest import golden_case, golden_meta
    from test_gpu_parity import make_model
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel

    def _run(nm, sparse, debug_steps=None):
        meta, gold = golden_case(nm)
        os.environ['WRNN_SPARSE'] = '1' if sparse else '0'
        m, hp, sd = make_model(meta)
        m.set_engine('persist')
        if debug_steps:
            m.set_debug_steps(debug_steps)
        mel = synth_mel(meta['n_frames'], meta['mel_seed']) / sp.max_abs_value
        wav = m.generate(mel[None], meta['batched'], meta['target'], meta['overlap'], hp.mu_law,
                         sp.preemphasize, progress_callback=lambda *a: None)
        return meta, gold, m, wav

    for nm in sorted(k for k, v in golden_meta().items() if v.get('prune')):
        _run(nm, True)
    meta, gold = golden_case(name)
    steps = [int(s) for s in gold['logits_steps']][:4]
    rows = range(meta['num_folds'])
    bad = 0
    for i in range(int(n)):
        _, _, ms, _ = _run(name, True, steps)
        _, _, md, _ = _run(name, False, steps)
        a = np.stack([ms.debug_logits(s, rows) for s in steps])
        b = np.stack([md.debug_logits(s, rows) for s in steps])
        d = np.argwhere(a.view(np.uint32) != b.view(np.uint32))
        if len(d):
            bad += 1
            ref = gold['logits'][:len(steps)]
            ea = np.abs(a.astype(np.float64) - ref).max(axis=2)
            eb = np.abs(b.astype(np.float64) - ref).max(axis=2)
            ent = sorted({(int(x), int(y)) for x, y, _ in d})
            print(f'rep {i}: labels equal {np.array_equal(ms.last_labels, md.last_labels)}; differing (step idx, row) '
                  f'{ent}; sparse err {[float(ea[x, y]) for x, y in ent]} dense err {[float(eb[x, y]) for x, y in ent]}',
                  flush=True)
        del ms, md
    print(f'{bad} of {n} repetitions differ', flush=True)


if __name__ == '__main__':
    main(*sys.argv[1:])
