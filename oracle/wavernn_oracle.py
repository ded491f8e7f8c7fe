"""CPU oracle: a functional torch-CPU / numpy restatement of the reference WaveRNN generate().

TEST INFRASTRUCTURE ONLY. Only tests/, tests/golden/gen_golden.py, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module, and only as the checker (or as the
timed CPU baseline). The MI355X product path never calls it and fails loudly when its HIP
library is missing.

What it restates (same torch ops, same order, same fp32/f64 dtypes as the reference):

* ``WaveRNN.generate``          vocoder/models/fatchord_version.py:155-259
                                vocoder/models/runtimeracer_version.py:199-314
                                vocoder/models/geneing_version.py:157-253 (I, rnn1, fc1, fc3;
                                2-way aux split; BITS = categorical over 2**bits, no mu-law;
                                RAW = Beta(exp(l0), exp(l1)) on the Philox BETA contract)
* ``UpsampleNetwork.forward``   fatchord_version.py:78-85 (+ MelResNet :38-44, ResBlock :17-24,
                                Stretch2d :53-57); runtimeracer_version.py:88-95
* ``pad_tensor``                fatchord_version.py:275-288
* ``fold_with_overlap``         fatchord_version.py:290-340
* ``xfade_and_unfold``          fatchord_version.py:342-404
* ``get_gru_cell``/GRUCell      fatchord_version.py:267-273 -> torch.gru_cell (same ATen op)
* RAW sampler                   fatchord_version.py:225-228: softmax -> Categorical(p).sample()
                                == argmax((p / p.sum()) / q), q ~ Exp(1) (torch 2.10 multinomial
                                single-sample fast path); q is injected from oracle.philox.
* MOL sampler                   vocoder/distribution.py:104-140 with the two ``uniform_``
                                draws injected from oracle.philox.
* decode_mu_law / de_emphasis   vocoder/audio.py:102-107, :92-93 (scipy lfilter)
* fade-out                      fatchord_version.py:252-255

Parity pin: tests/golden/gen_golden.py runs the real reference generate() in the survey
container with the same injected noise and commits its outputs; tests/test_oracle_golden.py
checks this restatement reproduces them bit-for-bit.
"""
import math
import time

import numpy as np
import torch
import torch.nn.functional as F
from scipy.signal import lfilter

from oracle import philox

MODEL_TYPE_FATCHORD = 'fatchord-wavernn'
MODEL_TYPE_RUNTIMERACER = 'runtimeracer-wavernn'
MODEL_TYPE_GENEING = 'geneing-wavernn'


def _t(sd, name):
    v = sd[name]
    if isinstance(v, np.ndarray):
        v = torch.from_numpy(v)
    return v


class OracleWaveRNN:
    """Holds torch-CPU tensors of one WaveRNN state dict; no nn.Module."""

    def __init__(self, sd, hp, model_type, hop_length=200, feat_dims=80):
        self.sd = {k: _t(sd, k) for k in sd}
        self.hp = hp
        self.model_type = model_type
        self.mode = hp.mode
        self.pad = hp.pad
        # geneing_version.py:95-101: 'RAW' = the 2 parameters of a Beta distribution
        self.beta = model_type == MODEL_TYPE_GENEING and hp.mode == 'RAW'
        self.n_classes = 2 if self.beta else 2 ** hp.bits if hp.mode in ('RAW', 'BITS') else 30
        self.rnn_dims = hp.rnn_dims
        # geneing_version.py:106 splits the aux into 2 parts, the others into 4
        self.n_aux = 2 if model_type == MODEL_TYPE_GENEING else 4
        self.aux_dims = hp.res_out_dims // self.n_aux
        self.hop_length = hop_length
        self.upsample_factors = tuple(hp.upsample_factors)
        self.indent = hp.pad * int(np.cumprod(self.upsample_factors)[-1])
        self.total_scale = int(np.cumprod(self.upsample_factors)[-1])

    # --- upsample network (fatchord_version.py:9-85) -------------------------------
    def _bn(self, x, p):
        s = self.sd
        return F.batch_norm(x, s[p + '.running_mean'], s[p + '.running_var'], s[p + '.weight'],
                            s[p + '.bias'], False, 0.1, 1e-5)

    def resnet(self, x):
        s = self.sd
        x = F.conv1d(x, s['upsample.resnet.conv_in.weight'], None)
        x = self._bn(x, 'upsample.resnet.batch_norm')
        x = F.relu(x)
        for i in range(self.hp.res_blocks):
            p = f'upsample.resnet.layers.{i}'
            residual = x
            x = F.conv1d(x, s[p + '.conv1.weight'], None)
            x = self._bn(x, p + '.batch_norm1')
            x = F.relu(x)
            x = F.conv1d(x, s[p + '.conv2.weight'], None)
            x = self._bn(x, p + '.batch_norm2')
            x = x + residual
        x = F.conv1d(x, s['upsample.resnet.conv_out.weight'], s['upsample.resnet.conv_out.bias'])
        return x

    @staticmethod
    def stretch2d(x, x_scale, y_scale):
        b, c, h, w = x.size()
        x = x.unsqueeze(-1).unsqueeze(3)
        x = x.repeat(1, 1, 1, y_scale, 1, x_scale)
        return x.view(b, c, h * y_scale, w * x_scale)

    def upsample(self, m):
        aux = self.resnet(m).unsqueeze(1)
        aux = self.stretch2d(aux, self.total_scale, 1)
        aux = aux.squeeze(1)
        m = m.unsqueeze(1)
        for j, scale in enumerate(self.upsample_factors):
            m = self.stretch2d(m, scale, 1)
            m = F.conv2d(m, self.sd[f'upsample.up_layers.{2 * j + 1}.weight'], None, 1, (0, scale))
        m = m.squeeze(1)[:, :, self.indent:-self.indent]
        return m.transpose(1, 2), aux.transpose(1, 2)

    # --- fold helpers (fatchord_version.py:275-404) ---------------------------------
    @staticmethod
    def pad_tensor(x, pad, side='both'):
        b, t, c = x.size()
        total = t + 2 * pad if side == 'both' else t + pad
        padded = torch.zeros(b, total, c)
        if side == 'before' or side == 'both':
            padded[:, pad:pad + t, :] = x
        elif side == 'after':
            padded[:, :t, :] = x
        return padded

    def fold_with_overlap(self, x, target, overlap):
        _, total_len, features = x.size()
        num_folds = (total_len - overlap) // (target + overlap)
        extended_len = num_folds * (overlap + target) + overlap
        remaining = total_len - extended_len
        if remaining != 0:
            num_folds += 1
            padding = target + 2 * overlap - remaining
            x = self.pad_tensor(x, padding, side='after')
        folded = torch.zeros(num_folds, target + 2 * overlap, features)
        for i in range(num_folds):
            start = i * (target + overlap)
            end = start + target + 2 * overlap
            folded[i] = x[:, start:end, :]
        return folded

    @staticmethod
    def xfade_and_unfold(y, target, overlap):
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

    # --- one recurrent step (fatchord :194-213 / runtimeracer :244-270) -------------
    def _gru(self, name, x, h):
        s = self.sd
        return torch.gru_cell(x, h, s[name + '.weight_ih_l0'], s[name + '.weight_hh_l0'],
                              s[name + '.bias_ih_l0'], s[name + '.bias_hh_l0'])

    def _lin(self, name, x):
        return F.linear(x, self.sd[name + '.weight'], self.sd[name + '.bias'])

    def step(self, x, hs, m_t, a_t):
        if self.model_type == MODEL_TYPE_GENEING:  # geneing_version.py:193-205
            a1_t, a2_t = a_t
            x = torch.cat([x, m_t, a1_t[:, :-1]], dim=1)
            x = self._lin('I', x)
            h1, = hs
            h1 = self._gru('rnn1', x, h1)
            x = x + h1
            x = torch.cat([x, a2_t], dim=1)
            x = F.relu(self._lin('fc1', x))
            logits = self._lin('fc3', x)
            return logits, (h1,)
        a1_t, a2_t, a3_t, a4_t = a_t
        x = torch.cat([x, m_t, a1_t[:, :-1]], dim=1)
        x = self._lin('I', x)
        if self.model_type == MODEL_TYPE_FATCHORD:
            h1, h2 = hs
            h1 = self._gru('rnn1', x, h1)
            x = x + h1
            inp = torch.cat([x, a2_t], dim=1)
            h2 = self._gru('rnn2', inp, h2)
            x = x + h2
            x = torch.cat([x, a3_t], dim=1)
            x = F.relu(self._lin('fc1', x))
            x = torch.cat([x, a4_t], dim=1)
            x = F.relu(self._lin('fc2', x))
            logits = self._lin('fc3', x)
            return logits, (h1, h2)
        h1, h2, h3, h4 = hs
        h1 = self._gru('rnn1', x, h1)
        x = x + h1
        h2 = self._gru('rnn2', x, h2)
        x = x + h2
        inp = torch.cat([x, a2_t], dim=1)
        h3 = self._gru('rnn3', inp, h3)
        x = x + h3
        h4 = self._gru('rnn4', x, h4)
        x = x + h4
        x = torch.cat([x, a3_t], dim=1)
        x = self._lin('fc1', x)
        x = F.relu(self._lin('fc2', x))
        x = torch.cat([x, a4_t], dim=1)
        x = self._lin('fc3', x)
        x = F.relu(self._lin('fc4', x))
        logits = self._lin('fc5', x)
        return logits, (h1, h2, h3, h4)

    # --- samplers --------------------------------------------------------------------
    def sample_raw(self, logits, q, gaps=None):
        """fatchord_version.py:225-228 with Categorical.sample() == argmax(probs / q).
        ``gaps``: a list that receives, per row, the decision's top-1 / top-2 gap
        log(r1) - log(r2) of the fp32 ratios r = probs / q (how far the draw was from a flip)."""
        posterior = F.softmax(logits, dim=1)
        probs = posterior / posterior.sum(-1, keepdim=True)   # Categorical.__init__
        ratio = probs / q
        k = torch.argmax(ratio, dim=-1)                       # multinomial fast path
        sample = 2 * k.float() / (self.n_classes - 1.) - 1.
        if gaps is not None:
            top = torch.topk(ratio, 2, dim=-1).values.double().numpy()
            gaps.append(np.log(top[:, 0]) - np.log(top[:, 1]))
        return k, sample

    @staticmethod
    def sample_mol(y, u1, u2, log_scale_min=None):
        """vocoder/distribution.py:104-140 with the uniform_ draws replaced by (u1, u2)."""
        if log_scale_min is None:
            log_scale_min = float(np.log(1e-14))
        nr_mix = y.size(1) // 3
        y = y.transpose(1, 2)
        logit_probs = y[:, :, :nr_mix]
        temp = u1
        temp = logit_probs.data - torch.log(- torch.log(temp))
        _, argmax = temp.max(dim=-1)
        one_hot = torch.FloatTensor(argmax.size() + (nr_mix,)).zero_()
        one_hot.scatter_(len(argmax.size()), argmax.unsqueeze(-1), 1.)
        means = torch.sum(y[:, :, nr_mix:2 * nr_mix] * one_hot, dim=-1)
        log_scales = torch.clamp(torch.sum(y[:, :, 2 * nr_mix:3 * nr_mix] * one_hot, dim=-1),
                                 min=log_scale_min)
        u = u2
        x = means + torch.exp(log_scales) * (torch.log(u) - torch.log(1. - u))
        x = torch.clamp(torch.clamp(x, min=-1.), max=1.)
        return x, argmax

    # --- generate ----------------------------------------------------------------------
    def prepare(self, mels, batched, target, overlap):
        """Steps :166-190: pad, upsample, fold. Returns (mels_f, aux_f, wave_len)."""
        wave_len = (mels.size(-1) - 1) * self.hop_length
        mels = self.pad_tensor(mels.transpose(1, 2), pad=self.pad, side='both')
        mels, aux = self.upsample(mels.transpose(1, 2))
        if batched:
            mels = self.fold_with_overlap(mels, target, overlap)
            aux = self.fold_with_overlap(aux, target, overlap)
        return mels, aux, wave_len

    def generate(self, mels, batched, target, overlap, mu_law, apply_preemphasis, seed=0,
                 stream=0, max_steps=None, progress_callback=None, record_logits=None,
                 post=True, track_margin=False):
        """Restates generate(); returns a dict with 'wav' and per-row outputs.

        ``mels``: torch (1, n_mels, T) float32, already divided by max_abs_value.
        ``max_steps``: stop the recurrence early (bounded CPU-baseline sample); 'wav' is
        then None.
        ``post=False``: rows only, no post-processing ('wav' None) -- mels shorter than the
        20-hop tail fade have rows but no waveform (the reference raises there, :253-255).
        ``record_logits``: optional list of step indices whose logits are returned.
        ``track_margin``: RAW only -- 'margin' = the smallest top-1 / top-2 gap (log of the fp32
        probs / q ratios) over every (step, row) decision, with its step and row.
        """
        mu_law = mu_law if self.mode == 'RAW' else False  # geneing BITS: no mu-law (:158)
        start = time.time()
        out = {}
        with torch.no_grad():
            t0 = time.time()
            mels, aux, wave_len = self.prepare(mels, batched, target, overlap)
            out['t_prepare'] = time.time() - t0
            b_size, seq_len, _ = mels.size()
            n_steps = seq_len if max_steps is None else min(seq_len, max_steps)
            n_gru = {MODEL_TYPE_FATCHORD: 2, MODEL_TYPE_GENEING: 1}.get(self.model_type, 4)
            hs = tuple(torch.zeros(b_size, self.rnn_dims) for _ in range(n_gru))
            x = torch.zeros(b_size, 1)
            d = self.aux_dims
            aux_split = [aux[:, :, d * i:d * (i + 1)] for i in range(self.n_aux)]
            rows = np.arange(b_size)
            labels = np.zeros((b_size, n_steps), dtype=np.int16)
            samples = []
            logits_rec = {}
            margin = [math.inf, -1, -1]
            t0 = time.time()
            for i in range(n_steps):
                m_t = mels[:, i, :]
                a_t = tuple(a[:, i, :] for a in aux_split)
                logits, hs = self.step(x, hs, m_t, a_t)
                if record_logits is not None and i in record_logits:
                    logits_rec[i] = logits.clone().numpy()
                if self.beta:
                    # vocoder/distribution.py:7-20 with Beta(alpha, beta).sample() on the
                    # Philox BETA contract: alpha, beta = exp(logits) in fp32
                    loc = logits.exp()
                    sample = torch.from_numpy(philox.beta_sample(
                        seed, stream, i, rows, loc[:, 0].numpy(), loc[:, 1].numpy()))
                    samples.append(sample)
                    x = sample.unsqueeze(-1)
                elif self.mode == 'MOL':
                    u1, u2 = philox.mol_uniforms(seed, stream, [i], rows)
                    sample, _ = self.sample_mol(logits.unsqueeze(0).transpose(1, 2),
                                                torch.from_numpy(u1), torch.from_numpy(u2))
                    samples.append(sample.view(-1))
                    x = sample.transpose(0, 1)
                else:
                    q = torch.from_numpy(philox.raw_exp_noise(seed, stream, [i], rows,
                                                              self.n_classes)[0])
                    g = [] if track_margin else None
                    k, sample = self.sample_raw(logits, q, g)
                    if g:
                        j = int(np.argmin(g[0]))
                        if g[0][j] < margin[0]:
                            margin[:] = [float(g[0][j]), i, j]
                    labels[:, i] = k.numpy().astype(np.int16)
                    samples.append(sample)
                    x = sample.unsqueeze(-1)
                if progress_callback is not None and i % 100 == 0:
                    gen_rate = (i + 1) / (time.time() - start) * b_size / 1000
                    progress_callback(i, seq_len, b_size, gen_rate)
            out['t_loop'] = time.time() - t0
        out['B'], out['S'], out['steps'] = b_size, seq_len, n_steps
        out['labels'] = labels if self.mode != 'MOL' and not self.beta else None
        output = torch.stack(samples).transpose(0, 1)
        out['samples'] = output.numpy().copy()
        out['logits'] = logits_rec
        if track_margin and margin[1] >= 0:
            out['margin'] = {'min_gap': margin[0], 'step': margin[1], 'row': margin[2]}
        if n_steps < seq_len or not post:
            out['wav'] = None
            return out
        t0 = time.time()
        output = output.cpu().numpy().astype(np.float64)
        if batched:
            output = self.xfade_and_unfold(output, target, overlap)
        else:
            output = output[0]
        if mu_law:
            output = decode_mu_law(output, self.n_classes, False)
        if apply_preemphasis:
            output = de_emphasis(output)
        fade_out = np.linspace(1, 0, 20 * self.hop_length)
        output = output[:wave_len]
        output[-20 * self.hop_length:] *= fade_out
        out['t_post'] = time.time() - t0
        out['wav'] = output
        return out


def label_2_float(x, bits):
    return 2 * x / (2 ** bits - 1.) - 1.


def decode_mu_law(y, mu, from_labels=True):
    """vocoder/audio.py:102-107."""
    if from_labels:
        y = label_2_float(y, math.log2(mu))
    mu = mu - 1
    x = np.sign(y) / mu * ((1 + mu) ** np.abs(y) - 1)
    return x


def de_emphasis(x, preemphasis=0.97):
    """vocoder/audio.py:92-93."""
    return lfilter([1], [1, -preemphasis], x)


def oracle_infer_waveform(sd, hp, model_type, mel, normalize=True, batched=True, target=None,
                          overlap=None, seed=0, stream=0, max_abs_value=4., preemphasize=True,
                          **kw):
    """vocoder/inference.py:59-95 around OracleWaveRNN.generate."""
    if target is None:
        target = hp.gen_target
    if overlap is None:
        overlap = hp.gen_overlap
    if normalize:
        mel = mel / max_abs_value
    mel = torch.from_numpy(mel[None, ...])
    model = OracleWaveRNN(sd, hp, model_type)
    return model.generate(mel, batched, target, overlap, hp.mu_law, preemphasize, seed=seed,
                          stream=stream, **kw)
