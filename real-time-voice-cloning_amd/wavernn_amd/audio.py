"""Host-side f64 post-processing of the vocoder output (restated from the reference).

* ``label_2_float``  vocoder/audio.py:9-10
* ``decode_mu_law``  vocoder/audio.py:102-107
* ``de_emphasis``    vocoder/audio.py:92-93 (scipy.signal.lfilter, same call)
* ``xfade_and_unfold`` vocoder/models/fatchord_version.py:342-404
* ``fade_out_tail``  vocoder/models/fatchord_version.py:252-255

These run on the host in float64 exactly as the reference does (same numpy/scipy calls in the
same order), so given identical per-fold samples the waveform is bit-identical.
"""
import math

import numpy as np
from scipy.signal import lfilter

from .hparams import sp


def label_2_float(x, bits):
    return 2 * x / (2 ** bits - 1.) - 1.


def labels_to_samples(labels, n_classes):
    """torch ``2 * k.float() / (n_classes - 1.) - 1.`` in fp32 (fatchord_version.py:228)."""
    k = labels.astype(np.float32)
    return (np.float32(2) * k) / np.float32(n_classes - 1.) - np.float32(1.)


def decode_mu_law(y, mu, from_labels=True):
    if from_labels:
        y = label_2_float(y, math.log2(mu))
    mu = mu - 1
    x = np.sign(y) / mu * ((1 + mu) ** np.abs(y) - 1)
    return x


def encode_mu_law(x, mu):
    mu = mu - 1
    fx = np.sign(x) * np.log(1 + mu * np.abs(x)) / np.log(1 + mu)
    return np.floor((fx + 1) / 2 * mu + 0.5)


def de_emphasis(x):
    return lfilter([1], [1, -sp.preemphasis], x)


def de_emphasis_native(x, lib):
    """de_emphasis through the library's host loop (wrnn_de_emphasis: scipy's lfilter
    recurrence, same doubles), without scipy's generic filter machinery."""
    import ctypes
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty_like(x)
    pd = ctypes.POINTER(ctypes.c_double)
    rc = lib.wrnn_de_emphasis(x.ctypes.data_as(pd), y.ctypes.data_as(pd), x.size,
                              float(sp.preemphasis))
    if rc:
        raise RuntimeError('wrnn_de_emphasis failed (%d)' % rc)
    return y


def pre_emphasis(x):
    return lfilter([1, -sp.preemphasis], [1], x)


def xfade_and_unfold(y, target, overlap):
    """Equal-power cross-fade of the fold rows, overlap-added into one signal (f64)."""
    num_folds, length = y.shape
    target = length - 2 * overlap
    total_len = num_folds * (target + overlap) + overlap
    silence_len = overlap // 2
    fade_len = overlap - silence_len
    silence = np.zeros((silence_len), dtype=np.float64)
    t = np.linspace(-1, 1, fade_len, dtype=np.float64)
    fade_in = np.sqrt(0.5 * (1 + t))
    fade_out = np.sqrt(0.5 * (1 - t))
    fade_in = np.concatenate([silence, fade_in])
    fade_out = np.concatenate([fade_out, silence])
    y[:, :overlap] *= fade_in
    y[:, -overlap:] *= fade_out
    unfolded = np.zeros((total_len), dtype=np.float64)
    for i in range(num_folds):
        start = i * (target + overlap)
        end = start + target + 2 * overlap
        unfolded[start:end] += y[i]
    return unfolded


def _mu_law_unfolded(unfolded, labels, overlap, n_classes):
    """decode_mu_law(unfolded, n_classes, False), element for element, for the output of
    xfade_and_unfold over categorical rows: each fold's middle `target` samples are its labels'
    values untouched (0 + v), so they are looked up in a table of the n_classes decoded label
    values (the same numpy expression on the same f64 inputs); only the cross-faded overlaps
    are decoded directly."""
    num_folds, length = labels.shape
    target = length - 2 * overlap
    lut = decode_mu_law(labels_to_samples(np.arange(n_classes), n_classes).astype(np.float64),
                        n_classes, False)
    out = np.empty_like(unfolded)
    out[:overlap] = decode_mu_law(unfolded[:overlap], n_classes, False)
    # after the first overlap, fold i owns [middle (target) | overlap with fold i + 1]
    u = unfolded[overlap:].reshape(num_folds, target + overlap)
    o = out[overlap:].reshape(num_folds, target + overlap)
    o[:, :target] = lut[labels[:, overlap:overlap + target].astype(np.intp)]
    o[:, target:] = decode_mu_law(u[:, target:], n_classes, False)
    return out


_POST_TABLES = {}


def _post_tables(n_classes, overlap, mu_law, fade_len):
    """Per-(n_classes, overlap, mu_law, fade_len) tables of the fused label path: the f64 value
    of every label, the middle-sample table (decoded if mu_law), xfade_and_unfold's fade_in /
    fade_out and the final fade, each built with the reference's own numpy expressions."""
    key = (n_classes, overlap, mu_law, fade_len)
    t = _POST_TABLES.get(key)
    if t is None:
        samp = labels_to_samples(np.arange(n_classes), n_classes).astype(np.float64)
        mid = decode_mu_law(samp, n_classes, False) if mu_law else samp.copy()
        silence_len = overlap // 2
        fade_len_x = overlap - silence_len
        tt = np.linspace(-1, 1, fade_len_x, dtype=np.float64)
        silence = np.zeros((silence_len), dtype=np.float64)
        fade_in = np.ascontiguousarray(np.concatenate([silence, np.sqrt(0.5 * (1 + tt))]))
        fade_out = np.ascontiguousarray(np.concatenate([np.sqrt(0.5 * (1 - tt)), silence]))
        fade = np.ascontiguousarray(np.linspace(1, 0, fade_len))
        t = _POST_TABLES[key] = (np.ascontiguousarray(samp), np.ascontiguousarray(mid),
                                 fade_in, fade_out, fade)
    return t


def postprocess_labels(labels, target, overlap, mu_law, apply_preemphasis, n_classes,
                       wave_len, hop_length, lib):
    """postprocess() for batched categorical rows (labels (nf, S) int16), fused in the
    library's host loops (wrnn_post_overlaps / wrnn_post_assemble): the same doubles as
    xfade_and_unfold -> decode_mu_law -> de_emphasis -> fade, without the full-length
    intermediates. Only the nf + 1 cross-faded overlap regions are decoded here, by the
    reference's numpy expression; the middles come from a table of decoded label values.
    Returns None when the shape is outside the fused path (the caller uses postprocess())."""
    labels = np.ascontiguousarray(labels, dtype=np.int16)
    nf, S = labels.shape
    fade_len = 20 * hop_length
    total = nf * (S - overlap) + overlap
    n_out = min(int(wave_len), total)
    if overlap < 1 or S < 2 * overlap + 1 or n_out < fade_len or wave_len < 0:
        return None
    samp, mid, fade_in, fade_out, fade = _post_tables(n_classes, overlap, bool(mu_law),
                                                      fade_len)
    regions = np.empty((nf + 1, overlap), np.float64)
    rc = lib.wrnn_post_overlaps(labels.ctypes.data, nf, S, overlap, samp.ctypes.data,
                                n_classes, fade_in.ctypes.data, fade_out.ctypes.data,
                                regions.ctypes.data)
    if rc:
        raise RuntimeError('wrnn_post_overlaps failed (%d)' % rc)
    if mu_law:
        regions = np.ascontiguousarray(decode_mu_law(regions, n_classes, False))
    out = np.empty(n_out, np.float64)
    rc = lib.wrnn_post_assemble(labels.ctypes.data, nf, S, overlap, mid.ctypes.data,
                                n_classes, regions.ctypes.data, int(bool(apply_preemphasis)),
                                float(sp.preemphasis), fade.ctypes.data, fade_len,
                                out.ctypes.data, n_out)
    if rc:
        raise RuntimeError('wrnn_post_assemble failed (%d)' % rc)
    return out


def postprocess(samples, batched, target, overlap, mu_law, apply_preemphasis, n_classes,
                wave_len, hop_length, labels=None, lib=None):
    """fatchord_version.py:238-255 on the (B, S) per-fold samples (any float dtype).
    ``labels``: the categorical rows the samples came from, if any (mu-law table path);
    ``lib``: the loaded C-ABI library, if any (native de-emphasis loop)."""
    if batched and labels is not None and lib is not None:
        out = postprocess_labels(labels, target, overlap, mu_law, apply_preemphasis, n_classes,
                                 wave_len, hop_length, lib)
        if out is not None:
            return out
    output = np.asarray(samples).astype(np.float64)
    if batched:
        output = xfade_and_unfold(output, target, overlap)
    else:
        output = output[0]
    if mu_law and batched and labels is not None and overlap > 0:
        output = _mu_law_unfolded(output, np.asarray(labels), overlap, n_classes)
    elif mu_law:
        output = decode_mu_law(output, n_classes, False)
    if apply_preemphasis:
        output = de_emphasis_native(output, lib) if lib is not None else de_emphasis(output)
    fade_out = np.linspace(1, 0, 20 * hop_length)
    output = output[:wave_len]
    output[-20 * hop_length:] *= fade_out
    return output
