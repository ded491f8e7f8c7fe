"""Seeded synthetic weights and mels with the reference's state-dict layout.

No trained checkpoint is available offline (the reference ships none), so
tests and the bench use random-init weights of the exact reference architecture. The
generator is numpy PCG64 so any machine (this container or a GPU box without the
reference) regenerates bit-identical tensors from a seed.

Key names and shapes follow the reference modules:
``vocoder/models/fatchord_version.py:9-118``, ``vocoder/models/geneing_version.py:88-120`` and
``vocoder/models/runtimeracer_version.py:98-137`` (``upsample.resnet.*``, ``upsample.up_layers.{1,3,5}.weight``, ``I``, ``rnn*``,
``fc*``, ``step``). Init ranges follow torch's defaults for those module types
(U(+-1/sqrt(fan_in)) for Linear/Conv, U(+-1/sqrt(hidden)) for GRU); BatchNorm statistics are
randomised so that folding and ordering bugs cannot hide behind the identity transform.
"""
import numpy as np

MODEL_TYPE_FATCHORD = 'fatchord-wavernn'
MODEL_TYPE_RUNTIMERACER = 'runtimeracer-wavernn'
MODEL_TYPE_GENEING = 'geneing-wavernn'


def n_classes_of(hp, model_type=None):
    """fc3 outputs: geneing 'RAW' = 2 Beta parameters (geneing_version.py:95-96), RAW / BITS
    = 2**bits classes, MOL = 30."""
    if model_type == MODEL_TYPE_GENEING and hp.mode == 'RAW':
        return 2
    return 2 ** hp.bits if hp.mode in ('RAW', 'BITS') else 30


def aux_dims_of(hp, model_type):
    """res_out_dims // 4 (fatchord, runtimeracer) or // 2 (geneing_version.py:106)."""
    return hp.res_out_dims // (2 if model_type == MODEL_TYPE_GENEING else 4)


def state_dict_spec(hp, model_type, feat_dims=80):
    """Ordered {name: shape} of the reference model's state_dict (minus BN counters)."""
    spec = {}
    C, R = hp.compute_dims, hp.res_out_dims
    k = hp.pad * 2 + 1
    spec['upsample.resnet.conv_in.weight'] = (C, feat_dims, k)
    for bn in ['upsample.resnet.batch_norm']:
        for f in ('weight', 'bias', 'running_mean', 'running_var'):
            spec[f'{bn}.{f}'] = (C,)
    for i in range(hp.res_blocks):
        p = f'upsample.resnet.layers.{i}'
        spec[f'{p}.conv1.weight'] = (C, C, 1)
        spec[f'{p}.conv2.weight'] = (C, C, 1)
        for bn in ('batch_norm1', 'batch_norm2'):
            for f in ('weight', 'bias', 'running_mean', 'running_var'):
                spec[f'{p}.{bn}.{f}'] = (C,)
    spec['upsample.resnet.conv_out.weight'] = (R, C, 1)
    spec['upsample.resnet.conv_out.bias'] = (R,)
    for j, s in enumerate(hp.upsample_factors):
        spec[f'upsample.up_layers.{2 * j + 1}.weight'] = (1, 1, 1, 2 * s + 1)
    H, F = hp.rnn_dims, hp.fc_dims
    A = aux_dims_of(hp, model_type)
    n = n_classes_of(hp, model_type)
    spec['I.weight'] = (H, feat_dims + A)
    spec['I.bias'] = (H,)

    def gru(name, inp):
        spec[f'{name}.weight_ih_l0'] = (3 * H, inp)
        spec[f'{name}.weight_hh_l0'] = (3 * H, H)
        spec[f'{name}.bias_ih_l0'] = (3 * H,)
        spec[f'{name}.bias_hh_l0'] = (3 * H,)

    def lin(name, inp, out):
        spec[f'{name}.weight'] = (out, inp)
        spec[f'{name}.bias'] = (out,)

    if model_type == MODEL_TYPE_FATCHORD:
        gru('rnn1', H)
        gru('rnn2', H + A)
        lin('fc1', H + A, F)
        lin('fc2', F + A, F)
        lin('fc3', F, n)
    elif model_type == MODEL_TYPE_GENEING:
        gru('rnn1', H)
        lin('fc1', H + A, F)
        lin('fc3', F, n)
    elif model_type == MODEL_TYPE_RUNTIMERACER:
        gru('rnn1', H)
        gru('rnn2', H)
        gru('rnn3', H + A)
        gru('rnn4', H)
        lin('fc1', H + A, F)
        lin('fc2', F, F)
        lin('fc3', F + A, F)
        lin('fc4', F, F)
        lin('fc5', F, n)
    else:
        raise NotImplementedError("Invalid model of type '%s' provided. Aborting..." % model_type)
    return spec


def _fan_in(name, shape):
    if len(shape) == 1:
        return None
    return int(np.prod(shape[1:]))


def synth_state_dict(hp, model_type, seed=0, logit_scale=1.0, feat_dims=80, gru_scale=1.0,
                     fc_scale=1.0):
    """Deterministic float32 weights {name: ndarray} (plus ``step``) for a topology.

    ``logit_scale`` scales the output layer (fatchord/geneing fc3, runtimeracer fc5),
    ``gru_scale`` every GRU parameter and ``fc_scale`` the hidden fc layers: the knobs that move
    the seeded init towards a trained checkpoint's statistics (saturated gates, peaked posteriors;
    tests/golden/gen_golden.py 'trained-like' fixtures). Scaling happens after the draws, so
    the other tensors do not depend on the knobs."""
    rng = np.random.Generator(np.random.PCG64(seed))
    spec = state_dict_spec(hp, model_type, feat_dims)
    sd = {}
    H = hp.rnn_dims
    for name, shape in spec.items():
        leaf = name.rsplit('.', 1)[-1]
        if 'up_layers' in name:
            k = shape[-1]
            w = (1.0 / k) * (1.0 + 0.1 * rng.uniform(-1.0, 1.0, size=shape))
        elif leaf == 'running_mean':
            w = rng.uniform(-0.2, 0.2, size=shape)
        elif leaf == 'running_var':
            w = rng.uniform(0.5, 1.5, size=shape)
        elif 'batch_norm' in name and leaf == 'weight':
            w = rng.uniform(0.8, 1.2, size=shape)
        elif 'batch_norm' in name and leaf == 'bias':
            w = rng.uniform(-0.1, 0.1, size=shape)
        elif name.startswith('rnn'):
            b = 1.0 / np.sqrt(H)
            w = rng.uniform(-b, b, size=shape)
        else:
            if leaf == 'bias':
                wshape = spec[name[:-len('bias')] + 'weight']
                fan = int(np.prod(wshape[1:]))
            else:
                fan = _fan_in(name, shape)
            b = 1.0 / np.sqrt(fan)
            w = rng.uniform(-b, b, size=shape)
        sd[name] = np.ascontiguousarray(w, dtype=np.float32)
    last_fc = 'fc5' if model_type == MODEL_TYPE_RUNTIMERACER else 'fc3'
    if logit_scale != 1.0:
        sd[f'{last_fc}.weight'] = (sd[f'{last_fc}.weight'] * np.float32(logit_scale)).astype(np.float32)
        sd[f'{last_fc}.bias'] = (sd[f'{last_fc}.bias'] * np.float32(logit_scale)).astype(np.float32)
    for name in list(sd):
        scale = (gru_scale if name.startswith('rnn') else
                 fc_scale if name.startswith('fc') and not name.startswith(last_fc + '.') else 1.0)
        if scale != 1.0:
            sd[name] = (sd[name] * np.float32(scale)).astype(np.float32)
    sd['step'] = np.zeros((1,), dtype=np.int64)
    return sd


def synth_mel(n_frames, seed=0, n_mels=80):
    """Synthetic symmetric-range mel in [-4, 4] (synthesizer/audio.py:181-193), float32 (n_mels, T)."""
    rng = np.random.default_rng(seed)
    return rng.uniform(-4, 4, (n_mels, n_frames)).astype(np.float32)
