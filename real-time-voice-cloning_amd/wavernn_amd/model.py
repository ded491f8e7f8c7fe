"""WaveRNN facade over the MI355X library: same constructor and ``generate`` as the reference.

Mirrors ``vocoder/models/fatchord_version.py:88-259`` / ``runtimeracer_version.py:98-314``:
``WaveRNN(rnn_dims, fc_dims, bits, pad, upsample_factors, feat_dims, compute_dims, res_out_dims,
res_blocks, hop_length, sample_rate, mode)`` plus ``model_type`` (which of the two topologies),
``load_state_dict`` with the reference's state-dict names, and
``generate(mels, batched, target, overlap, mu_law, apply_preemphasis, progress_callback)``
returning the float64 waveform of ``(T - 1) * hop_length`` samples.

The whole recurrence (upsample network, conditioning, GRU/FC steps, sampling) runs on the GPU
through the C-ABI; only the reference's f64 post-processing (cross-fade, mu-law, de-emphasis,
fade-out; fatchord_version.py:238-255) runs on the host, restated bit-exactly in audio.py.
"""
import ctypes
import os
import sys
import time
import warnings

import numpy as np

from . import _abi
from .audio import labels_to_samples, postprocess, postprocess_labels

MODEL_TYPE_FATCHORD = 'fatchord-wavernn'
MODEL_TYPE_RUNTIMERACER = 'runtimeracer-wavernn'
MODEL_TYPE_GENEING = 'geneing-wavernn'
_MODEL_IDS = {MODEL_TYPE_FATCHORD: _abi.WRNN_MODEL_FATCHORD,
              MODEL_TYPE_RUNTIMERACER: _abi.WRNN_MODEL_RUNTIMERACER,
              MODEL_TYPE_GENEING: _abi.WRNN_MODEL_GENEING}


def _progbar(i, n, size=16):
    done = (i * size) // n
    return ''.join('█' if j <= done else '░' for j in range(size))


def _wrap_callback(progress_callback):
    """ctypes callback around the user's progress_callback: an exception it raises stops the
    call (non-zero return -> WRNN_ERR_ABORTED) and is re-raised by the caller afterwards
    (``err[0]``), as the reference's generate() would propagate it."""
    err = [None]
    if progress_callback is None:
        return _abi.PROGRESS_FN(), err

    def _cb(user, i, seq_len, b_size, rate):
        try:
            progress_callback(i, seq_len, b_size, rate)
        except BaseException as e:  # noqa: B902 -- surfaced after the native call
            err[0] = e
            return 1
        return 0
    return _abi.PROGRESS_FN(_cb), err


def _to_numpy_f32(x):
    if hasattr(x, 'detach'):
        x = x.detach().cpu().numpy()
    return np.ascontiguousarray(np.asarray(x, dtype=np.float32))


class WaveRNN:
    def __init__(self, rnn_dims, fc_dims, bits, pad, upsample_factors, feat_dims, compute_dims,
                 res_out_dims, res_blocks, hop_length, sample_rate, mode='RAW', pruning=False,
                 model_type=MODEL_TYPE_FATCHORD, device=0):
        if model_type not in _MODEL_IDS:
            raise NotImplementedError("Invalid model of type '%s' provided. Aborting..." % model_type)
        geneing = model_type == MODEL_TYPE_GENEING
        if geneing and mode == 'RAW':
            # geneing_version.py:95-96,207-210: 2 outputs, Beta(exp l0, exp l1) on [-1, 1]
            self.n_classes = 2
        elif mode == 'RAW' or (geneing and mode == 'BITS'):
            self.n_classes = 2 ** bits
        elif mode == 'MOL':
            self.n_classes = 30
        else:
            raise RuntimeError("Unknown model mode value - ", mode)
        # categorical sampling over n_classes: RAW (fatchord / runtimeracer) and geneing BITS;
        # continuous samples: MOL and geneing RAW (Beta)
        self.categorical = mode != 'MOL' and not (geneing and mode == 'RAW')
        self._dev_mode = (_abi.WRNN_MODE_RAW if self.categorical else
                          _abi.WRNN_MODE_BETA if mode == 'RAW' else _abi.WRNN_MODE_MOL)
        self.mode = mode
        self.bits = bits
        self.pad = pad
        self.rnn_dims = rnn_dims
        self.fc_dims = fc_dims
        self.aux_dims = res_out_dims // (2 if geneing else 4)
        self.hop_length = hop_length
        self.sample_rate = sample_rate
        self.model_type = model_type
        self.upsample_factors = tuple(upsample_factors)
        self.device = device
        self._step = 0
        self._lib = _abi.load_library()
        cfg = _abi.WrnnConfig()
        cfg.model_type = _MODEL_IDS[model_type]
        cfg.mode = self._dev_mode
        cfg.bits = bits
        cfg.rnn_dims, cfg.fc_dims = rnn_dims, fc_dims
        cfg.compute_dims, cfg.res_out_dims = compute_dims, res_out_dims
        cfg.res_blocks, cfg.pad = res_blocks, pad
        cfg.feat_dims, cfg.hop_length = feat_dims, hop_length
        cfg.n_upsample = len(self.upsample_factors)
        for i, s in enumerate(self.upsample_factors):
            cfg.upsample_factors[i] = s
        self._cfg = cfg
        h = ctypes.c_void_p()
        _abi.check(self._lib.wrnn_create(ctypes.byref(cfg), int(device), ctypes.byref(h)),
                   'wrnn_create')
        self._h = h
        self._loaded = False
        self.timings = {}

    def __del__(self):
        h = getattr(self, '_h', None)
        if h is not None and h.value:
            try:
                self._lib.wrnn_destroy(h)
            except Exception:
                pass
            self._h = None

    # --- torch.nn.Module-like surface used by the reference's callers -----------------
    def eval(self):
        return self

    def train(self, mode=True):
        return self

    def to(self, device):
        return self

    def get_step(self):
        return self._step

    def num_params(self, print_out=False):
        return None

    def load_state_dict(self, state_dict, strict=True):
        """Upload a reference state dict (torch tensors or numpy arrays, PyTorch layout)."""
        for name, value in state_dict.items():
            if name == 'step':
                self._step = int(np.asarray(value.cpu() if hasattr(value, 'cpu') else value)
                                 .reshape(-1)[0])
                continue
            if name.endswith('num_batches_tracked'):
                continue
            arr = _to_numpy_f32(value)
            shape = (ctypes.c_int64 * arr.ndim)(*arr.shape)
            _abi.check(self._lib.wrnn_load_tensor(
                self._h, name.encode(), arr.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                shape, arr.ndim), 'load_state_dict')
        _abi.check(self._lib.wrnn_finalize(self._h), 'load_state_dict')
        self._loaded = True

    def load_bin(self, data):
        """Load a libwavernn .bin weight file (path or bytes; vocoder/libwavernn/convert.py)."""
        if isinstance(data, (str, os.PathLike)):
            try:
                with open(data, 'rb') as f:
                    data = f.read()
            except OSError:
                raise RuntimeError("Cannot open file.")  # WaveRNNVocoder.cpp:24-26
        data = bytes(data)
        _abi.check(self._lib.wrnn_load_bin(self._h, data, len(data)), 'loadWeights')
        self._loaded = True

    def set_seed(self, seed):
        _abi.check(self._lib.wrnn_set_seed(self._h, ctypes.c_uint64(int(seed) & (2 ** 64 - 1))))

    def set_stream(self, stream):
        _abi.check(self._lib.wrnn_set_stream(self._h, ctypes.c_uint32(int(stream))))

    def get_stream(self):
        """Noise stream the next call's first utterance will use."""
        s = ctypes.c_uint32()
        _abi.check(self._lib.wrnn_get_stream(self._h, ctypes.byref(s)))
        return s.value

    def _set_utt_streams(self, streams, n_utts):
        if streams is None:
            return
        streams = [int(s) for s in streams]
        if len(streams) != n_utts:
            raise ValueError(f'{len(streams)} streams for {n_utts} utterances')
        arr = (ctypes.c_uint32 * len(streams))(*streams)
        _abi.check(self._lib.wrnn_set_utt_streams(self._h, arr, len(streams)))

    def _set_fold_ranges(self, ranges, n_utts):
        if ranges is None:
            return
        ranges = [(int(lo), int(hi)) for lo, hi in ranges]
        if len(ranges) != n_utts:
            raise ValueError(f'{len(ranges)} fold ranges for {n_utts} utterances')
        lo = (ctypes.c_int * n_utts)(*[r[0] for r in ranges])
        hi = (ctypes.c_int * n_utts)(*[r[1] for r in ranges])
        _abi.check(self._lib.wrnn_set_fold_ranges(self._h, lo, hi, n_utts))

    def fold_shape(self, n_frames, batched, target, overlap):
        b, s = ctypes.c_int(), ctypes.c_int()
        _abi.check(self._lib.wrnn_fold_shape(int(n_frames), self.hop_length, int(bool(batched)),
                                             int(target or 0), int(overlap or 0),
                                             ctypes.byref(b), ctypes.byref(s)))
        return b.value, s.value

    def set_engine(self, engine):
        """'auto' (default), 'chain' or 'persist' for later calls (include/wavernn_mi355x.h)."""
        if engine not in _abi.ENGINES:
            raise ValueError(f'unknown engine {engine!r}; expected one of {sorted(_abi.ENGINES)}')
        _abi.check(self._lib.wrnn_set_engine(self._h, _abi.ENGINES[engine]))

    def last_engine(self):
        """Engine ('chain' or 'persist') that ran the last call."""
        e = ctypes.c_int()
        _abi.check(self._lib.wrnn_last_engine(self._h, ctypes.byref(e)))
        return {v: k for k, v in _abi.ENGINES.items()}[e.value]

    def plan_info(self):
        """Launches of the last persistent call: [(first_row, rows_per_group, wide)]."""
        n = ctypes.c_int()
        cap = 64
        fr, nr, wd = (ctypes.c_int * cap)(), (ctypes.c_int * cap)(), (ctypes.c_int * cap)()
        _abi.check(self._lib.wrnn_plan_info(self._h, ctypes.byref(n), fr, nr, wd, cap))
        return [(fr[i], nr[i], bool(wd[i])) for i in range(min(n.value, cap))]

    def rot_info(self):
        """Row rotation of the last persistent call: (launches, steps per
        launch of the q + 1-row groups, of the q-row groups); (0, 0, 0) when none."""
        k, nh, nl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _abi.check(self._lib.wrnn_rot_info(self._h, ctypes.byref(k), ctypes.byref(nh), ctypes.byref(nl)))
        return k.value, nh.value, nl.value

    def persist_steps(self, stage):
        """Steps per launch of persistent stage `stage` (stage_info order) of the last call."""
        v = ctypes.c_double()
        _abi.check(self._lib.wrnn_persist_steps(self._h, int(stage), ctypes.byref(v)))
        return v.value

    def sparse_info(self):
        """Block-sparse execution (pruned checkpoints): dict(available,
        last_call, density, fill_f4) -- whether the loaded weights have a sparse image, whether
        the last call ran it, the live fraction of the step matrices' 1 x 4 blocks, and the
        fullest slot's LDS list size."""
        av, lc, fill = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        d = ctypes.c_double()
        _abi.check(self._lib.wrnn_sparse_info(self._h, ctypes.byref(av), ctypes.byref(lc),
                                              ctypes.byref(d), ctypes.byref(fill)))
        return dict(available=bool(av.value), last_call=bool(lc.value), density=d.value,
                    fill_f4=fill.value)

    def rates(self):
        """The launch planner's rate table in effect (text, first line its source)."""
        buf = ctypes.create_string_buffer(4096)
        _abi.check(self._lib.wrnn_get_rates(self._h, buf, 4096))
        return buf.value.decode()

    def set_rates(self, table=None):
        """Override keys of the planner's rate table (None: reload as at creation)."""
        _abi.check(self._lib.wrnn_set_rates(self._h, table.encode() if table else None))

    def fallback_info(self):
        """(calls that fell back from PERSIST to CHAIN on this handle, last reason)."""
        n = ctypes.c_int()
        why = ctypes.create_string_buffer(256)
        _abi.check(self._lib.wrnn_fallback_info(self._h, ctypes.byref(n), why, 256))
        return n.value, why.value.decode('utf-8', 'replace')

    def _warn_fallback(self, before):
        n, why = self.fallback_info()
        if n > before:
            warnings.warn(f'WaveRNN (MI355X): the persistent engine could not run ({why}); this '
                          f'call ran on the chain engine (~14x slower)', RuntimeWarning,
                          stacklevel=3)

    def enable_stage_timing(self, enable=True):
        _abi.check(self._lib.wrnn_enable_stage_timing(self._h, int(bool(enable))))

    def stage_info(self):
        """[(name, algorithmic bytes/launch, flops/launch, avg us, launches)] of the last call."""
        n = ctypes.c_int()
        name = ctypes.create_string_buffer(64)
        by, fl = ctypes.c_double(), ctypes.c_double()
        _abi.check(self._lib.wrnn_stage_info(self._h, 0, name, 64, ctypes.byref(by),
                                             ctypes.byref(fl), ctypes.byref(n)))
        out = []
        for s in range(n.value):
            _abi.check(self._lib.wrnn_stage_info(self._h, s, name, 64, ctypes.byref(by),
                                                 ctypes.byref(fl), None))
            us, cnt = ctypes.c_double(), ctypes.c_int()
            rc = self._lib.wrnn_stage_timing(self._h, s, ctypes.byref(us), ctypes.byref(cnt))
            out.append((name.value.decode(), by.value, fl.value,
                        us.value if rc == 0 else float('nan'), cnt.value if rc == 0 else 0))
        return out

    def debug_noise(self, n_steps, n_rows):
        """RAW Exp(1) noise of the last call, (n_steps, n_rows, n_classes) float32."""
        out = np.empty((n_steps, n_rows, self.n_classes), dtype=np.float32)
        _abi.check(self._lib.wrnn_debug_noise(self._h, n_steps,
                                              out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                              out.size))
        return out

    def debug_upsample(self, n_frames, feat_dims=80, res_out_dims=None):
        """(mel_up (feat, L), aux (res_out_dims, T)) of the last call's first utterance."""
        R = res_out_dims or self.aux_dims * 4
        L = n_frames * self.hop_length
        mel = np.empty((feat_dims, L), dtype=np.float32)
        aux = np.empty((R, n_frames), dtype=np.float32)
        fp = ctypes.POINTER(ctypes.c_float)
        _abi.check(self._lib.wrnn_debug_upsample(self._h, mel.ctypes.data_as(fp), mel.size,
                                                 aux.ctypes.data_as(fp), aux.size))
        return mel, aux

    def debug_p1(self, step, row):
        """PERSIST conditioning input of the last persistent call at (step, fold row):
        (rnn_dims, 4) float32 per unit: r, z, n of W_ih1 (I c) + b_ih1, then I c + b_I."""
        out = np.empty((self.rnn_dims, 4), dtype=np.float32)
        _abi.check(self._lib.wrnn_debug_p1(self._h, step, row,
                                           out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                           out.size))
        return out

    def set_debug_steps(self, steps):
        """Record the pre-sampling logits of every fold row at these steps (<= 8) in later
        calls; [] / None turns recording off (wrnn_set_debug_steps)."""
        steps = [int(s) for s in (steps or [])]
        arr = (ctypes.c_int * max(1, len(steps)))(*steps)
        _abi.check(self._lib.wrnn_set_debug_steps(self._h, arr, len(steps)))

    def debug_logits(self, step, rows):
        """Logits of the last call at a recorded step: (len(rows), n_classes) float32."""
        out = np.empty((len(rows), self.n_classes), dtype=np.float32)
        for i, r in enumerate(rows):
            _abi.check(self._lib.wrnn_debug_logits(
                self._h, int(step), int(r), out[i].ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                self.n_classes))
        return out

    def gen_display(self, i, seq_len, b_size, gen_rate):
        pbar = _progbar(i, seq_len)
        msg = f'| {pbar} {i*b_size}/{seq_len*b_size} | Batch Size: {b_size} | Gen Rate: {gen_rate:.1f}kHz | '
        sys.stdout.write(f"\r{msg}")

    # --- the hot path ------------------------------------------------------------------
    def generate_rows(self, mels, batched, target, overlap, progress_callback=None):
        """Device recurrence only: returns (labels or None, samples (B,S) f32, B, S)."""
        if not self._loaded:
            raise RuntimeError("Model hasn't been loaded. Call loadWeights first.")
        mel = _to_numpy_f32(mels)
        if mel.ndim == 3:
            mel = mel[0]
        mel = np.ascontiguousarray(mel)
        T = mel.shape[-1]
        B, S = self.fold_shape(T, batched, target, overlap)
        n = B * S
        labels = np.empty((B, S), dtype=np.int16) if self.categorical else None
        samples = None if self.categorical else np.empty((B, S), dtype=np.float32)
        cfn, cb_ref = _wrap_callback(progress_callback)
        ob, os_ = ctypes.c_int(), ctypes.c_int()
        fb0 = self.fallback_info()[0]
        rc = self._lib.wrnn_generate(
            self._h, mel.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), T,
            int(bool(batched)), int(target or 0), int(overlap or 0),
            labels.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)) if labels is not None else None,
            samples.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) if samples is not None else None,
            n, ctypes.byref(ob), ctypes.byref(os_), cfn, None)
        if cb_ref[0] is not None:
            raise cb_ref[0]
        _abi.check(rc, 'generate')
        self._warn_fallback(fb0)
        if labels is not None:
            samples = labels_to_samples(labels, self.n_classes)
        return labels, samples, B, S

    def generate_batch_device(self, mels_dev, batched, target, overlap, progress_callback=None,
                              streams=None, fold_ranges=None):
        """Several utterances as one batch of fold rows, inputs resident in HBM.

        ``mels_dev``: list of torch CUDA float32 tensors (feat_dims, T_u) on this model's device
        (already normalised). Returns (out_dev, row_offset, S): ``out_dev`` is a torch CUDA
        tensor (rows, S) -- int16 labels (RAW) or float32 samples (MOL). ``streams``: explicit
        noise stream per utterance (default: the handle's counter + u; wrnn_set_utt_streams).
        ``fold_ranges``: [(lo, hi)] per utterance -- run only fold rows lo .. hi - 1 of it
        (wrnn_set_fold_ranges: the rows equal those of a full call bit for bit).
        """
        import torch
        if not self._loaded:
            raise RuntimeError("Model hasn't been loaded. Call loadWeights first.")
        n = len(mels_dev)
        for name, lst in (('streams', streams), ('fold ranges', fold_ranges)):
            if lst is not None and len(lst) != n:  # (before either list is armed on the handle)
                raise ValueError(f'{len(lst)} {name} for {n} utterances')
        mels_dev = [m.contiguous() for m in mels_dev]
        for m in mels_dev:
            if m.dtype != torch.float32 or not m.is_cuda:
                raise ValueError('mels must be float32 CUDA tensors')
        frames = (ctypes.c_int * n)(*[int(m.shape[-1]) for m in mels_dev])
        ptrs = (ctypes.c_void_p * n)(*[m.data_ptr() for m in mels_dev])
        rows = 0
        S = 0
        for u, m in enumerate(mels_dev):
            b, S = self.fold_shape(int(m.shape[-1]), batched, target, overlap)
            if fold_ranges is not None and u < len(fold_ranges):
                lo, hi = fold_ranges[u]
                b = max(0, min(int(hi), b) - max(int(lo), 0))
            rows += b
        dev = mels_dev[0].device
        if self.categorical:
            out = torch.empty((rows, S), dtype=torch.int16, device=dev)
            lab_p, smp_p = out.data_ptr(), None
        else:
            out = torch.empty((rows, S), dtype=torch.float32, device=dev)
            lab_p, smp_p = None, out.data_ptr()
        roff = (ctypes.c_int * (n + 1))()
        s_out = ctypes.c_int()
        cfn, cb_ref = _wrap_callback(progress_callback)
        torch.cuda.current_stream(dev).synchronize()
        fb0 = self.fallback_info()[0]
        self._set_utt_streams(streams, n)
        self._set_fold_ranges(fold_ranges, n)
        rc = self._lib.wrnn_generate_batch_device(
            self._h, n, ptrs, frames, int(bool(batched)), int(target or 0), int(overlap or 0),
            lab_p, smp_p, rows * S, roff, ctypes.byref(s_out), cfn, None)
        if cb_ref[0] is not None:
            raise cb_ref[0]
        _abi.check(rc, 'generate_batch_device')
        self._warn_fallback(fb0)
        return out, list(roff), S

    def generate_batch(self, mels_dev, batched, target, overlap, mu_law, apply_preemphasis,
                       progress_callback=None, streams=None):
        """generate() for several device-resident mels; returns a list of f64 waveforms."""
        mu_law = mu_law if self.mode == 'RAW' else False
        out, roff, S = self.generate_batch_device(mels_dev, batched, target, overlap,
                                                  progress_callback, streams=streams)
        host = out.cpu().numpy()
        self.last_batch_rows, self.last_batch_offsets = host, roff
        return [self.postprocess_rows(host[roff[u]:roff[u + 1]], int(m.shape[-1]), batched,
                                      target, overlap, mu_law, apply_preemphasis)
                for u, m in enumerate(mels_dev)]

    def postprocess_rows(self, rows, n_frames, batched, target, overlap, mu_law,
                         apply_preemphasis):
        """Host f64 post-processing of one utterance's fold rows (fatchord_version.py:238-255):
        ``rows`` (num_folds, S) int16 labels (categorical) or float32 samples (MOL, Beta)."""
        mu_law = mu_law if self.mode == 'RAW' else False
        wave_len = (int(n_frames) - 1) * self.hop_length
        if self.categorical and batched:
            wav = postprocess_labels(rows, target, overlap, mu_law, apply_preemphasis,
                                     self.n_classes, wave_len, self.hop_length, self._lib)
            if wav is not None:
                return wav
        smp = labels_to_samples(rows, self.n_classes) if self.categorical else rows
        return postprocess(smp, batched, target, overlap, mu_law, apply_preemphasis,
                           self.n_classes, wave_len, self.hop_length,
                           labels=rows if self.categorical else None, lib=self._lib)

    def generate(self, mels, batched, target, overlap, mu_law, apply_preemphasis,
                 progress_callback=None):
        """fatchord_version.py:155-259 (runtimeracer_version.py:199-314) on the MI355X."""
        mu_law = mu_law if self.mode == 'RAW' else False
        progress_callback = progress_callback or self.gen_display
        mel = _to_numpy_f32(mels)
        T = mel.shape[-1]
        wave_len = (T - 1) * self.hop_length
        t0 = time.time()
        labels, samples, B, S = self.generate_rows(mel, batched, target, overlap,
                                                   progress_callback)
        t1 = time.time()
        out = postprocess(samples, batched, target, overlap, mu_law, apply_preemphasis,
                          self.n_classes, wave_len, self.hop_length, labels=labels,
                          lib=self._lib)
        self.timings = dict(device=t1 - t0, post=time.time() - t1, B=B, S=S)
        self.last_labels = labels
        self.last_samples = samples
        return out
