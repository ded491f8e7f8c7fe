"""CPU: the per-frame form of the PERSIST conditioning (runtime.hip pack_p1). The mel upsampler
(three Stretch2d + 1 x (2s+1) conv stages, vocoder/models/fatchord_version.py:47-85) is linear
and, for every real frame, the same kernel shifted by hop, so mel_up(hop f + s) =
sum_k K[s][k] mel(f - 2 + k). This restates the derivation pack_p1 runs (unit impulses through
the stencil chain in float64, shift invariance checked on every frame) and checks the tap form
against the oracle's own torch upsample for random up-layer weights. The C++ code itself is
pinned on the GPU (tests/test_gpu_parity.py::test_persist_p1_matches_oracle)."""
import numpy as np
import pytest
import torch

from oracle.wavernn_oracle import OracleWaveRNN


def stencil_chain(x, ws, factors, pad, indent):
    """k_mel_stencil in float64 on a (T,) sequence; returns the trimmed upsampled sequence."""
    cur, in_pad, T_in, W_in = x, pad, len(x), len(x) + 2 * pad
    for st, (w, s) in enumerate(zip(ws, factors)):
        W_out = W_in * s
        last = st == len(factors) - 1
        lo, ln = (indent, W_out - 2 * indent) if last else (0, W_out)
        out = np.zeros(ln)
        for oo in range(ln):
            for d in range(2 * s + 1):
                i = lo + oo + d - s
                q = i // s - in_pad if 0 <= i < W_out else -1
                if 0 <= q < T_in:
                    out[oo] += w[d] * cur[q]
        cur, in_pad, T_in, W_in = out, 0, ln, ln
    return cur


@pytest.mark.parametrize('factors', [(5, 5, 8), (4, 5, 10)])
def test_tap_form_reproduces_the_upsampler(factors):
    rng = np.random.default_rng(7)
    hop, pad = int(np.prod(factors)), 2
    indent = pad * hop
    ws = [rng.uniform(0.5, 1.5, 2 * s + 1) for s in factors]
    Tt = 9
    resp = [stencil_chain(np.eye(Tt)[j], ws, factors, pad, indent) for j in range(Tt)]
    jm = Tt // 2

    def G(x):
        p = hop * jm + x
        return resp[jm][p] if 0 <= p < hop * Tt else 0.0

    for j in range(Tt):  # shift invariance on every frame, edges included
        for p in range(hop * Tt):
            assert abs(resp[j][p] - G(p - hop * j)) <= 1e-12 * (1 + abs(G(p - hop * j)))
    taps = np.array([[G(s + hop * (2 - k)) for k in range(5)] for s in range(hop)])
    # every phase needs at most 4 consecutive frames, starting at f - 2 below a split phase and
    # at f - 1 from it on (the in-kernel 4-tap form)
    split = next(c for c in range(hop + 1)
                 if all(taps[s, 4 if s < c else 0] == 0 for s in range(hop)))
    assert 0 < split < hop
    # against the reference's own upsample (the oracle: torch Stretch2d + conv2d in fp32)
    T = 23
    mel = rng.uniform(-1, 1, (80, T)).astype(np.float32)
    hp = type('hp', (), {'pad': pad, 'upsample_factors': factors, 'mode': 'RAW', 'bits': 9,
                         'rnn_dims': 512, 'res_out_dims': 128})()
    sd = {f'upsample.up_layers.{2 * j + 1}.weight': torch.tensor(w, dtype=torch.float32).view(1, 1, 1, -1)
          for j, w in enumerate(ws)}
    o = OracleWaveRNN(sd, hp, 'fatchord-wavernn', hop_length=hop)
    m = torch.from_numpy(mel)[None]
    padded = torch.nn.functional.pad(m, (pad, pad))
    x = padded.unsqueeze(1)
    for j, s in enumerate(factors):
        x = o.stretch2d(x, s, 1)
        x = torch.nn.functional.conv2d(x, sd[f'upsample.up_layers.{2 * j + 1}.weight'], None, 1, (0, s))
    ref = x.squeeze(1)[0, :, indent:-indent].double().numpy()  # (80, hop T)
    mp = np.zeros((80, T + 4))
    mp[:, 2:T + 2] = mel
    rec = np.zeros_like(ref)
    for p in range(hop * T):
        f, s = divmod(p, hop)
        rec[:, p] = mp[:, f:f + 5] @ taps[s]  # frames f - 2 .. f + 2 = padded f .. f + 4
    scale = np.abs(ref).max()
    assert np.abs(rec - ref).max() <= 2e-6 * scale
