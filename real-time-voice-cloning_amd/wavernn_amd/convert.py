"""libwavernn ``.bin`` weight files: writer and reader.

Mirrors ``vocoder/libwavernn/convert.py`` of the reference (``convert_model`` :14-58, the
1x4 block compression :60-81, the per-layer records :83-156, the layer order :303-351) so a
checkpoint can be turned into the file the reference's C++ vocoder loads, and such a file can be
loaded back into this build (``wrnn_bin_read`` / ``wrnn_load_bin`` in the C-ABI do the parsing;
``read_bin`` here is a thin ctypes wrapper around the former, host only).

The writer works from a state dict (numpy or torch tensors), not from ``nn.Module`` objects;
the module repr that the reference stores in each 64-byte layer name field is informational
(the C++ reader skips it) and is written as the module's class name here.

``el_size`` 2 writes every layer's arrays as IEEE binary16 (the reference's ``elSize = 4
#change to 2 for fp16``, convert.py:12); the reader widens them to fp32 on load. The
BatchNorm eps stays fp32 as in the reference's ``'@iif'`` record.
"""
import ctypes
import struct
from pathlib import Path

import numpy as np

from . import _abi
from .hparams import sp

LAYER_IDS = {'Conv1d': 1, 'Conv2d': 2, 'BatchNorm1d': 3, 'Linear': 4, 'GRU': 5, 'Stretch2d': 6}
EL_SIZE = 4
SPARSE_GROUP = 4  # hparams.sparse_group


def _np(x):
    if hasattr(x, 'detach'):
        x = x.detach().cpu().numpy()
    return np.ascontiguousarray(np.asarray(x, dtype=np.float32))


def compress(W, group=SPARSE_GROUP):
    """(weights of the non-zero 1xgroup blocks, uint8 index stream) -- convert.py:60-74."""
    W = _np(W)
    rows, cols = W.shape
    blocks = (W.reshape(rows, cols // group, group) != 0).any(axis=-1)
    idx = []
    for r in range(rows):
        idx.extend(np.nonzero(blocks[r])[0].tolist())
        idx.append(255)
    idx.append(255)  # the reference's loop runs one row past the end
    keep = np.repeat(blocks, group, axis=1)
    return W[keep], np.asarray(idx, dtype=np.uint8)


class _Writer:
    def __init__(self, f, el_size=EL_SIZE):
        if el_size not in (4, 2):
            raise ValueError('el_size must be 4 (fp32) or 2 (fp16)')
        self.f = f
        self.el = el_size

    def raw(self, fmt, *v):
        self.f.write(struct.pack(fmt, *v))

    def arr(self, a, name=''):
        a = _np(a)
        if self.el == 2:
            with np.errstate(over='ignore'):
                h = a.astype(np.float16)
            # a finite value past the fp16 range would be written as inf: refuse the file
            bad = np.isfinite(a) & ~np.isfinite(h)
            if bad.any():
                raise ValueError(f'{name or "array"}: {int(bad.sum())} value(s) outside the fp16 range '
                                 f'(|x| > 65504, e.g. {float(a[bad][0])}); write this model with '
                                 f'el_size=4')
            a = h
        self.f.write(a.tobytes(order='C'))

    def layer(self, kind, name):
        self.raw('@i64s', LAYER_IDS[kind], name.encode()[:64])

    def compressed(self, W, name=''):
        w, idx = compress(W)
        self.raw('@i', w.size)
        self.arr(w, name)
        self.raw('@i', idx.size)
        self.f.write(idx.tobytes(order='C'))

    def conv1d(self, sd, p, bias):
        W = _np(sd[p + '.weight'])
        out_ch, in_ch, k = W.shape
        self.layer('Conv1d', 'Conv1d')
        self.raw('@iiiii', self.el, int(bias), in_ch, out_ch, k)
        self.arr(W, p + '.weight')
        if bias:
            self.arr(sd[p + '.bias'], p + '.bias')

    def batchnorm(self, sd, p, eps=1e-5):
        w = _np(sd[p + '.weight'])
        self.layer('BatchNorm1d', 'BatchNorm1d')
        self.raw('@iif', self.el, w.size, eps)
        for f in ('weight', 'bias', 'running_mean', 'running_var'):
            self.arr(sd[f'{p}.{f}'], f'{p}.{f}')

    def linear(self, sd, p):
        W = _np(sd[p + '.weight'])
        self.layer('Linear', 'Linear')
        self.raw('@iii', self.el, W.shape[0], W.shape[1])
        self.compressed(W, p + '.weight')
        self.arr(sd[p + '.bias'], p + '.bias')

    def gru(self, sd, p):
        wih, whh = _np(sd[p + '.weight_ih_l0']), _np(sd[p + '.weight_hh_l0'])
        bih, bhh = _np(sd[p + '.bias_ih_l0']), _np(sd[p + '.bias_hh_l0'])
        H = whh.shape[1]
        self.layer('GRU', 'GRU')
        self.raw('@iii', self.el, H, wih.shape[1])
        for W in (*np.vsplit(wih, 3), *np.vsplit(whh, 3)):
            self.compressed(W, p + '.weight')
        for b in (*np.split(bih, 3), *np.split(bhh, 3)):
            self.arr(b, p + '.bias')

    def stretch(self, x, y):
        self.layer('Stretch2d', 'Stretch2d')
        self.raw('@ii', x, y)


def write_bin(f, state_dict, hp, model_type, el_size=EL_SIZE):
    """Write ``state_dict`` of a ``model_type`` WaveRNN with hparams ``hp`` as a .bin stream
    (arrays fp32 for ``el_size`` 4, fp16 for 2)."""
    from .model import MODEL_TYPE_FATCHORD, MODEL_TYPE_GENEING, MODEL_TYPE_RUNTIMERACER
    sd = state_dict
    w = _Writer(f, el_size)
    scale = int(np.prod(hp.upsample_factors))
    w.raw('@iiii', hp.res_blocks, len(hp.upsample_factors), scale, hp.pad)
    r = 'upsample.resnet'
    w.conv1d(sd, r + '.conv_in', False)
    w.batchnorm(sd, r + '.batch_norm')
    for i in range(hp.res_blocks):
        p = f'{r}.layers.{i}'
        w.conv1d(sd, p + '.conv1', False)
        w.batchnorm(sd, p + '.batch_norm1')
        w.conv1d(sd, p + '.conv2', False)
        w.batchnorm(sd, p + '.batch_norm2')
    w.conv1d(sd, r + '.conv_out', True)
    w.stretch(scale, 1)
    for j, s in enumerate(hp.upsample_factors):
        w.stretch(s, 1)
        k = _np(sd[f'upsample.up_layers.{2 * j + 1}.weight']).reshape(-1)
        w.layer('Conv2d', 'Conv2d')
        w.raw('@ii', w.el, k.size)
        w.arr(k, f'upsample.up_layers.{2 * j + 1}.weight')
    w.linear(sd, 'I')
    if model_type == MODEL_TYPE_FATCHORD:
        grus, fcs = ('rnn1', 'rnn2'), ('fc1', 'fc2', 'fc3')
    elif model_type == MODEL_TYPE_GENEING:  # convert.py:336-340
        grus, fcs = ('rnn1',), ('fc1', 'fc3')
    elif model_type == MODEL_TYPE_RUNTIMERACER:
        grus, fcs = ('rnn1', 'rnn2', 'rnn3', 'rnn4'), ('fc1', 'fc2', 'fc3', 'fc4', 'fc5')
    else:
        raise NotImplementedError("Invalid model of type '%s' provided. Aborting..." % model_type)
    for g in grus:
        w.gru(sd, g)
    for fc in fcs:
        w.linear(sd, fc)


def convert_model(model_fpath, default_model_type, out_dir, el_size=EL_SIZE):
    """convert.py:14-58: checkpoint (``torch.load(weights_only=True)``) -> ``out_dir/<stem>.bin``."""
    import torch
    from .base import hparams_for
    ckpt = torch.load(model_fpath, map_location='cpu', weights_only=True)
    model_type = ckpt.get('model_type', default_model_type)
    hp = hparams_for(model_type)
    out = Path(out_dir).joinpath(Path(model_fpath).stem).with_suffix('.bin')
    with open(out, 'wb') as f:
        write_bin(f, ckpt['model_state'], hp, model_type, el_size)
    return out


def config_for(hp, model_type):
    """The C-ABI topology struct of (hparams, model type)."""
    from .model import _MODEL_IDS
    cfg = _abi.WrnnConfig()
    cfg.model_type = _MODEL_IDS[model_type]
    from .model import MODEL_TYPE_GENEING
    cfg.mode = (_abi.WRNN_MODE_MOL if hp.mode == 'MOL' else
                _abi.WRNN_MODE_BETA if (model_type == MODEL_TYPE_GENEING and hp.mode == 'RAW') else
                _abi.WRNN_MODE_RAW)
    cfg.bits = hp.bits
    cfg.rnn_dims, cfg.fc_dims = hp.rnn_dims, hp.fc_dims
    cfg.compute_dims, cfg.res_out_dims = hp.compute_dims, hp.res_out_dims
    cfg.res_blocks, cfg.pad = hp.res_blocks, hp.pad
    cfg.feat_dims, cfg.hop_length = sp.num_mels, sp.hop_size
    cfg.n_upsample = len(hp.upsample_factors)
    for i, s in enumerate(hp.upsample_factors):
        cfg.upsample_factors[i] = s
    return cfg


def read_bin(data, hp, model_type):
    """Parse a .bin image with the library's reader (host only): {name: float32 array}."""
    lib = _abi.load_library()
    buf = bytes(data)
    out = {}

    def _put(user, name, ptr, shape, ndim):
        shp = tuple(shape[i] for i in range(ndim))
        n = int(np.prod(shp)) if shp else 1
        out[name.decode()] = np.ctypeslib.as_array(ptr, shape=(n,)).reshape(shp).copy()
        return 0

    cb = _abi.TENSOR_FN(_put)
    cfg = config_for(hp, model_type)
    _abi.check(lib.wrnn_bin_read(buf, len(buf), ctypes.byref(cfg), cb, None), 'read_bin')
    return out
