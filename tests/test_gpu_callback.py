"""progress_callback contract of WaveRNN.generate on both engines.

Reference: fatchord_version.py:234-236 calls ``progress_callback(i, seq_len, b_size, gen_rate)``
when ``i % 100 == 0`` -- so i = 0, 100, ..., in order, once each, b_size = number of fold rows.
On PERSIST the kernels publish their step count to host-mapped memory and the host reports from
it while one launch per row batch runs all steps (the callback no longer splits launches).
"""
import os

import numpy as np
import pytest

from conftest import golden_case

pytestmark = pytest.mark.gpu


def _model(name):
    from test_gpu_parity import make_model
    meta, gold = golden_case(name)
    m, hp, sd = make_model(meta)
    return meta, gold, m, hp


@pytest.mark.parametrize('engine', ['persist', 'chain'])
def test_callback_sequence_single_utterance(engine):
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    meta, gold, m, hp = _model('fatchord_raw9_config1')
    m.set_engine(engine)
    calls = []
    mel = synth_mel(meta['n_frames'], meta['mel_seed']) / sp.max_abs_value
    wav = m.generate(mel[None], True, meta['target'], meta['overlap'], hp.mu_law, sp.preemphasize,
                     progress_callback=lambda *c: calls.append(c))
    assert m.last_engine() == engine
    S, B = meta['seq_len'], meta['num_folds']
    assert [c[0] for c in calls] == list(range(0, S, 100))
    assert all(c[1] == S and c[2] == B and c[3] > 0 for c in calls)
    assert np.array_equal(wav, gold['wav'])


def test_callback_sequence_over_row_batches():
    """40 rows -> several persistent row batches: still i = 0, 100, ... < S exactly once."""
    import torch
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    meta, gold, m, hp = _model('fatchord_raw9_tiny')
    m.set_engine('persist')
    mels = [torch.from_numpy((synth_mel(meta['n_frames'], 300 + u) / sp.max_abs_value)
                             .astype(np.float32)).cuda() for u in range(8)]
    calls = []
    out, roff, S = m.generate_batch_device(mels, True, meta['target'], meta['overlap'],
                                           progress_callback=lambda *c: calls.append(c))
    assert m.last_engine() == 'persist'
    assert [c[0] for c in calls] == list(range(0, S, 100))
    assert all(c[1] == S and c[2] == roff[-1] for c in calls)


@pytest.mark.parametrize('engine', ['persist', 'chain'])
def test_callback_exception_propagates(engine):
    """An exception raised by the callback reaches the caller (as it would from the reference's
    Python loop) and no further callbacks run."""
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    meta, gold, m, hp = _model('fatchord_raw9_tiny')
    m.set_engine(engine)
    calls = []

    class Stop(Exception):
        pass

    def cb(i, *a):
        calls.append(i)
        if i >= 200:
            raise Stop()
    mel = synth_mel(meta['n_frames'], meta['mel_seed']) / sp.max_abs_value
    with pytest.raises(Stop):
        m.generate(mel[None], True, meta['target'], meta['overlap'], hp.mu_law, sp.preemphasize,
                   progress_callback=cb)
    assert calls == [0, 100, 200]
    # the handle stays usable
    m.set_seed(meta['noise_seed'])
    wav = m.generate(mel[None], True, meta['target'], meta['overlap'], hp.mu_law, sp.preemphasize,
                     progress_callback=lambda *a: None)
    assert np.array_equal(wav, gold['wav'])


def test_no_fallback_recorded():
    meta, gold, m, hp = _model('fatchord_raw9_tiny')
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    mel = synth_mel(meta['n_frames'], meta['mel_seed']) / sp.max_abs_value
    m.generate(mel[None], True, meta['target'], meta['overlap'], hp.mu_law, sp.preemphasize,
               progress_callback=lambda *a: None)
    assert m.last_engine() == 'persist'
    assert m.fallback_info()[0] == 0


def test_callbacks_arrive_while_the_launch_runs():
    """Progress is live: the first callback arrives long before the one persistent
    launch of a 12,100-step call has finished, and an exception raised at i = 200 stops the
    launch within ~100 steps instead of letting it run all S steps (the reference stops at the
    raising step)."""
    import time
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    meta, gold, m, hp = _model('fatchord_raw9_config1')
    m.set_engine('persist')
    mel = synth_mel(meta['n_frames'], meta['mel_seed']) / sp.max_abs_value
    run = lambda cb: m.generate(mel[None], True, meta['target'], meta['overlap'], hp.mu_law,
                                sp.preemphasize, progress_callback=cb)
    run(lambda *a: None)  # warm
    stamps = []
    t0 = time.perf_counter()
    run(lambda i, *a: stamps.append((i, time.perf_counter() - t0)))
    t_full = m.timings['device']
    assert stamps[0][0] == 0 and stamps[0][1] < 0.5 * t_full, (stamps[:2], t_full)
    # the callback times follow the steps (not all bunched at the end)
    mid = [t for i, t in stamps if i == 6000][0]
    assert stamps[0][1] < mid < stamps[-1][1]

    class Stop(Exception):
        pass

    def cb(i, *a):
        if i >= 200:
            raise Stop()
    t0 = time.perf_counter()
    with pytest.raises(Stop):
        run(cb)
    t_abort = time.perf_counter() - t0
    assert t_abort < 0.5 * t_full, (t_abort, t_full)
    m.set_seed(meta['noise_seed'])
    assert np.array_equal(run(lambda *a: None), gold['wav'])  # still usable, same result


@pytest.fixture(params=['1', 'occupancy'])
def persist_fails(request):
    """'1': a co-residency error preset in the launches' error word (they exit at
    registration); 'occupancy': the launch wrapper's occupancy check refuses the launch."""
    os.environ['WRNN_DEBUG_PERSIST_FAIL'] = request.param
    yield request.param
    os.environ.pop('WRNN_DEBUG_PERSIST_FAIL', None)


def test_persist_failure_falls_back_counted_and_warned(persist_fails):
    """A persistent launch that cannot run (injected co-residency failure at registration, or
    refused by the occupancy check before launching):
    AUTO reruns the call on CHAIN with the same result, counts it, warns, reports 'chain';
    an explicit 'persist' engine returns the error instead, at once."""
    import time
    meta, gold, m, hp = _model('fatchord_raw9_tiny')
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    mel = synth_mel(meta['n_frames'], meta['mel_seed']) / sp.max_abs_value
    with pytest.warns(RuntimeWarning, match='persistent engine could not run'):
        wav = m.generate(mel[None], True, meta['target'], meta['overlap'], hp.mu_law,
                         sp.preemphasize, progress_callback=lambda *a: None)
    assert np.array_equal(wav, gold['wav'])
    assert m.last_engine() == 'chain'
    n, why = m.fallback_info()
    assert n == 1 and 'co-resident' in why
    if persist_fails == 'occupancy':
        assert 'occupancy' in why
    m.set_engine('persist')
    m.set_seed(meta['noise_seed'])
    t0 = time.perf_counter()
    with pytest.raises(RuntimeError, match='co-resident'):
        m.generate(mel[None], True, meta['target'], meta['overlap'], hp.mu_law, sp.preemphasize,
                   progress_callback=lambda *a: None)
    assert time.perf_counter() - t0 < 0.5  # no 1 s spin
    # AUTO gives up only after kPersistMaxStreak failed calls in a row: a healthy call
    # afterwards runs persistent again
    os.environ.pop('WRNN_DEBUG_PERSIST_FAIL')
    m.set_engine('auto')
    m.set_seed(meta['noise_seed'])
    wav = m.generate(mel[None], True, meta['target'], meta['overlap'], hp.mu_law, sp.preemphasize,
                     progress_callback=lambda *a: None)
    assert m.last_engine() == 'persist'
    assert np.array_equal(wav, gold['wav'])
