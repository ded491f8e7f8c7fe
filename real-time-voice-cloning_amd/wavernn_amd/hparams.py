"""Hyper-parameters of the vocoder path, with the reference's names and values.

Mirrors ``config/hparams.py`` of the reference: the ``HParams`` container (:7-29, including
the comma-separated ``parse`` override), the signal-processing block ``sp`` (:38-51) and the
three WaveRNN topologies this build runs, ``wavernn_fatchord`` (:220-285),
``wavernn_geneing`` (:288-354) and ``wavernn_runtimeracer`` (:356-421). Only the fields the inference path reads are kept;
training-schedule, pruning and anomaly-detection fields are out of scope.
"""
import ast
import copy
import pprint


class HParams(object):
    """Attribute bag with ``parse("a=1,b=(5,5,8)")`` overrides (config/hparams.py:7-29)."""

    def __init__(self, **kwargs):
        self.__dict__.update(kwargs)

    def __setitem__(self, key, value):
        setattr(self, key, value)

    def __getitem__(self, key):
        return getattr(self, key)

    def __repr__(self):
        return pprint.pformat(self.__dict__)

    def parse(self, string):
        if len(string) > 0:
            overrides = [s.split("=") for s in string.split(",")]
            keys, values = zip(*overrides)
            keys = list(map(str.strip, keys))
            values = list(map(str.strip, values))
            for k in keys:
                self.__dict__[k] = ast.literal_eval(values[keys.index(k)])
        return self

    def copy(self, **overrides):
        hp = copy.deepcopy(self)
        hp.__dict__.update(overrides)
        return hp


# config/hparams.py:38-51
sp = HParams(
    sample_rate=16000,
    n_fft=1024,
    num_mels=80,
    hop_size=200,
    win_size=800,
    fmin=40,
    fmax=8000,
    min_level_db=-100,
    ref_level_db=20,
    max_abs_value=4.,
    preemphasis=0.97,
    preemphasize=True,
)

# config/hparams.py:220-285 (inference fields)
wavernn_fatchord = HParams(
    mode='RAW',
    bits=10,
    mu_law=True,
    upsample_factors=(5, 5, 8),
    rnn_dims=512,
    fc_dims=512,
    compute_dims=128,
    res_out_dims=32 * 4,
    res_blocks=10,
    pad=2,
    gen_batched=True,
    gen_target=3000,
    gen_overlap=1500,
)

# config/hparams.py:356-421 (inference fields)
wavernn_runtimeracer = HParams(
    mode='RAW',
    bits=10,
    mu_law=True,
    upsample_factors=(5, 5, 8),
    rnn_dims=256,
    fc_dims=256,
    compute_dims=128,
    res_out_dims=64 * 2,
    res_blocks=10,
    pad=2,
    gen_batched=True,
    gen_target=6000,
    gen_overlap=1000,
)

# config/hparams.py:288-354 (inference fields); mode 'BITS' = softmax over 2**bits classes
wavernn_geneing = HParams(
    mode='BITS',
    bits=10,
    mu_law=False,
    upsample_factors=(4, 5, 10),
    rnn_dims=256,
    fc_dims=128,
    compute_dims=64,
    res_out_dims=32 * 2,
    res_blocks=3,
    pad=2,
    gen_batched=True,
    gen_target=3000,
    gen_overlap=1500,
)
