"""Tacotron (SV2TTS) inference on PyTorch-ROCm.

Architecture and state-dict names follow the reference's ``synthesizer/models/tacotron.py``
(Encoder :12-60, CBHG :63-141, PreNet :143-157, LSA attention :179-216, Decoder :219-299,
Tacotron :302-450) and ``synthesizer/models/common_layers.py`` (HighwayNetwork :23-35,
BatchNormConv :38-50), so a reference checkpoint's ``model_state`` loads unchanged
(``torch.load(..., weights_only=True)``). Only the inference path (``generate``) is built.

The reference applies dropout in the prenets at inference too (``F.dropout(..., training=True)``,
tacotron.py:150-157), i.e. the synthesizer is stochastic. ``set_dropout_stream(seed)`` replaces
torch's RNG there with a reproducible mask stream (``DropoutStream``) so runs can be compared
against the reference on the same masks (tests/golden/gen_e2e_golden.py patches the reference
with the same stream); without it the torch RNG is used, as in the reference.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


class DropoutStream:
    """Deterministic prenet dropout masks: call i draws U[0,1) from PCG64([seed, i]) and keeps
    the elements >= p, scaled like torch's dropout (``x * (keep / (1 - p))``)."""

    def __init__(self, seed):
        self.seed = int(seed)
        self.calls = 0

    def __call__(self, x, p):
        rng = np.random.Generator(np.random.PCG64([self.seed, self.calls]))
        self.calls += 1
        keep = torch.from_numpy((rng.random(tuple(x.shape)) >= p).astype(np.float32)).to(x.device)
        return x * (keep / (1.0 - p))


_dropout = None  # None: torch's own dropout (the reference's behaviour)


def set_dropout_stream(seed):
    """Install (seed) or remove (None) the deterministic prenet dropout stream."""
    global _dropout
    _dropout = None if seed is None else DropoutStream(seed)


def prenet_dropout(x, p):
    if _dropout is not None:
        return _dropout(x, p)
    return F.dropout(x, p, training=True)


class _StaticMasks:
    """Prenet dropout inside a captured decoder chunk: call i multiplies by slot i of a device
    buffer that is refilled (from the mask stream) before every replay."""

    def __init__(self, buf):
        self.buf = buf  # list of (B, dims) tensors, in call order
        self.i = 0

    def __call__(self, x, p):
        m = self.buf[self.i]
        self.i += 1
        return x * m


class BatchNormConv(nn.Module):
    """conv (no bias, 'same' padding) -> optional ReLU -> BatchNorm (common_layers.py:38-50)."""

    def __init__(self, cin, cout, k, relu=True):
        super().__init__()
        self.conv = nn.Conv1d(cin, cout, k, stride=1, padding=k // 2, bias=False)
        self.bnorm = nn.BatchNorm1d(cout)
        self.relu = relu

    def forward(self, x):
        y = self.conv(x)
        return self.bnorm(F.relu(y) if self.relu else y)


class HighwayNetwork(nn.Module):
    """y = sigmoid(W2 x) * relu(W1 x) + (1 - sigmoid(W2 x)) * x (common_layers.py:23-35)."""

    def __init__(self, size):
        super().__init__()
        self.W1 = nn.Linear(size, size)
        self.W2 = nn.Linear(size, size)

    def forward(self, x):
        h = F.relu(self.W1(x))
        g = torch.sigmoid(self.W2(x))
        return g * h + (1. - g) * x


class CBHG(nn.Module):
    """1-D conv bank (k = 1..K) -> max-pool -> 2 projections + residual -> highways ->
    bidirectional GRU (tacotron.py:63-141)."""

    def __init__(self, K, in_channels, channels, proj_channels, num_highways):
        super().__init__()
        self.conv1d_bank = nn.ModuleList([BatchNormConv(in_channels, channels, k) for k in range(1, K + 1)])
        self.maxpool = nn.MaxPool1d(kernel_size=2, stride=1, padding=1)
        self.conv_project1 = BatchNormConv(K * channels, proj_channels[0], 3)
        self.conv_project2 = BatchNormConv(proj_channels[0], proj_channels[1], 3, relu=False)
        self.highway_mismatch = proj_channels[-1] != channels
        if self.highway_mismatch:
            self.pre_highway = nn.Linear(proj_channels[-1], channels, bias=False)
        self.highways = nn.ModuleList([HighwayNetwork(channels) for _ in range(num_highways)])
        self.rnn = nn.GRU(channels, channels // 2, batch_first=True, bidirectional=True)

    def forward(self, x):
        T = x.size(-1)
        bank = torch.cat([conv(x)[:, :, :T] for conv in self.conv1d_bank], dim=1)
        y = self.maxpool(bank)[:, :, :T]
        y = self.conv_project2(self.conv_project1(y)) + x
        y = y.transpose(1, 2)
        if self.highway_mismatch:
            y = self.pre_highway(y)
        for hw in self.highways:
            y = hw(y)
        self.rnn.flatten_parameters()
        return self.rnn(y)[0]


class PreNet(nn.Module):
    def __init__(self, in_dims, fc1_dims=256, fc2_dims=128, dropout=0.5):
        super().__init__()
        self.fc1 = nn.Linear(in_dims, fc1_dims)
        self.fc2 = nn.Linear(fc1_dims, fc2_dims)
        self.p = dropout

    def forward(self, x):
        x = prenet_dropout(F.relu(self.fc1(x)), self.p)
        return prenet_dropout(F.relu(self.fc2(x)), self.p)


class Encoder(nn.Module):
    """Character embedding -> prenet -> CBHG, then the speaker embedding tiled onto every
    character (SV2TTS, tacotron.py:12-60)."""

    def __init__(self, embed_dims, num_chars, encoder_dims, K, num_highways, dropout):
        super().__init__()
        self.embedding = nn.Embedding(num_chars, embed_dims)
        self.pre_net = PreNet(embed_dims, encoder_dims, encoder_dims, dropout)
        self.cbhg = CBHG(K, encoder_dims, encoder_dims, [encoder_dims, encoder_dims], num_highways)

    def forward(self, chars, speaker_embedding=None):
        x = self.pre_net(self.embedding(chars)).transpose(1, 2)
        x = self.cbhg(x)
        if speaker_embedding is None:
            return x
        B, N = x.size(0), x.size(1)
        e = speaker_embedding.reshape(B, -1)
        return torch.cat((x, e.unsqueeze(1).expand(B, N, e.size(1))), 2)


class LSA(nn.Module):
    """Location-sensitive attention over the cumulative alignment (tacotron.py:179-216)."""

    def __init__(self, attn_dim, kernel_size=31, filters=32):
        super().__init__()
        self.conv = nn.Conv1d(1, filters, padding=(kernel_size - 1) // 2, kernel_size=kernel_size, bias=True)
        self.L = nn.Linear(filters, attn_dim, bias=False)
        self.W = nn.Linear(attn_dim, attn_dim, bias=True)
        self.v = nn.Linear(attn_dim, 1, bias=False)
        self.cumulative = None

    def forward(self, enc_proj, query, t, chars):
        if t == 0:
            self.cumulative = torch.zeros(enc_proj.size(0), enc_proj.size(1), device=enc_proj.device)
        loc = self.L(self.conv(self.cumulative.unsqueeze(1)).transpose(1, 2))
        u = self.v(torch.tanh(self.W(query).unsqueeze(1) + enc_proj + loc)).squeeze(-1)
        u = u * (chars != 0).float()  # padding characters
        scores = F.softmax(u, dim=1)
        self.cumulative = self.cumulative + scores
        return scores.unsqueeze(1)


class Decoder(nn.Module):
    max_r = 20

    def __init__(self, n_mels, encoder_dims, decoder_dims, lstm_dims, dropout, spk_dims):
        super().__init__()
        self.register_buffer("r", torch.tensor(1, dtype=torch.int))
        self.n_mels = n_mels
        self.prenet = PreNet(n_mels, 2 * decoder_dims, 2 * decoder_dims, dropout)
        self.attn_net = LSA(decoder_dims)
        self.attn_rnn = nn.GRUCell(encoder_dims + 2 * decoder_dims + spk_dims, decoder_dims)
        self.rnn_input = nn.Linear(encoder_dims + decoder_dims + spk_dims, lstm_dims)
        self.res_rnn1 = nn.LSTMCell(lstm_dims, lstm_dims)
        self.res_rnn2 = nn.LSTMCell(lstm_dims, lstm_dims)
        self.mel_proj = nn.Linear(lstm_dims, n_mels * self.max_r, bias=False)
        self.stop_proj = nn.Linear(encoder_dims + spk_dims + lstm_dims, 1)

    def forward(self, enc, enc_proj, prenet_in, state, context, t, chars, r=None):
        """One decoder iteration (tacotron.py:244-299, eval mode: no zoneout). ``r``: the
        reduction factor as a host int (read from the buffer when absent)."""
        attn_h, h1, h2, c1, c2 = state
        attn_in = torch.cat([context, self.prenet(prenet_in)], dim=-1)
        attn_h = self.attn_rnn(attn_in.squeeze(1), attn_h)
        scores = self.attn_net(enc_proj, attn_h, t, chars)
        context = (scores @ enc).squeeze(1)
        x = self.rnn_input(torch.cat([context, attn_h], dim=1))
        h1, c1 = self.res_rnn1(x, (h1, c1))
        x = x + h1
        h2, c2 = self.res_rnn2(x, (h2, c2))
        x = x + h2
        r = int(self.r) if r is None else r
        mels = self.mel_proj(x).view(x.size(0), self.n_mels, self.max_r)[:, :, :r]
        stop = torch.sigmoid(self.stop_proj(torch.cat((x, context), dim=1)))
        return mels, scores, (attn_h, h1, h2, c1, c2), context, stop


class Tacotron(nn.Module):
    def __init__(self, embed_dims, num_chars, encoder_dims, decoder_dims, n_mels, fft_bins,
                 postnet_dims, encoder_K, lstm_dims, postnet_K, num_highways, dropout,
                 stop_threshold, speaker_embedding_size):
        super().__init__()
        self.n_mels = n_mels
        self.lstm_dims = lstm_dims
        self.encoder_dims = encoder_dims
        self.decoder_dims = decoder_dims
        self.speaker_embedding_size = speaker_embedding_size
        self.encoder = Encoder(embed_dims, num_chars, encoder_dims, encoder_K, num_highways, dropout)
        self.encoder_proj = nn.Linear(encoder_dims + speaker_embedding_size, decoder_dims, bias=False)
        self.decoder = Decoder(n_mels, encoder_dims, decoder_dims, lstm_dims, dropout, speaker_embedding_size)
        self.postnet = CBHG(postnet_K, n_mels, postnet_dims, [postnet_dims, fft_bins], num_highways)
        self.post_proj = nn.Linear(postnet_dims, fft_bins, bias=False)
        self.register_buffer("step", torch.zeros(1, dtype=torch.long))
        self.register_buffer("stop_threshold", torch.tensor(stop_threshold, dtype=torch.float32))

    @property
    def r(self):
        return int(self.decoder.r.item())

    @r.setter
    def r(self, value):
        self.decoder.r = self.decoder.r.new_tensor(value, requires_grad=False)

    def get_step(self):
        return int(self.step.item())

    def load(self, path, optimizer=None, checkpoint=None):
        if checkpoint is None:
            checkpoint = torch.load(str(path), map_location=next(self.parameters()).device,
                                    weights_only=True)
        self.load_state_dict(checkpoint["model_state"])

    @torch.no_grad()
    def generate(self, x, speaker_embedding=None, steps=2000, graph=None):
        """tacotron.py:393-450: returns (mel_outputs, postnet linear (B, fft_bins, T), attention).

        ``graph`` (default: on a GPU): run the decoder loop as replays of a captured HIP graph of
        ``GRAPH_CHUNK`` iterations (the eager loop is launch-bound: ~30 small kernels per
        iteration). Same kernels in the same order as the eager loop, same masks (the dropout
        stream is advanced exactly as the eager loop would), same stop rule: the outputs equal
        the eager ones."""
        self.eval()
        if graph is None:
            graph = x.is_cuda
        if graph:
            return self._generate_graph(x, speaker_embedding, steps)
        dev = next(self.parameters()).device
        B = x.size(0)
        z = lambda n: torch.zeros(B, n, device=dev)  # noqa: E731
        state = (z(self.decoder_dims), z(self.lstm_dims), z(self.lstm_dims), z(self.lstm_dims),
                 z(self.lstm_dims))
        context = z(self.encoder_dims + self.speaker_embedding_size)
        enc = self.encoder(x, speaker_embedding)
        enc_proj = self.encoder_proj(enc)
        mel_outputs, attn = [], []
        prenet_in = z(self.n_mels)
        for t in range(0, steps, self.r):
            mels, scores, state, context, stop = self.decoder(enc, enc_proj, prenet_in, state,
                                                              context, t, x)
            mel_outputs.append(mels)
            attn.append(scores)
            prenet_in = mels[:, :, -1]
            if (stop > 0.5).all() and t > 10:
                break
        mel_outputs = torch.cat(mel_outputs, dim=2)
        linear = self.post_proj(self.postnet(mel_outputs)).transpose(1, 2)
        return mel_outputs, linear, torch.cat(attn, 1)

    GRAPH_CHUNK = 32

    def _generate_graph(self, x, speaker_embedding, steps):
        global _dropout
        dev = x.device
        B, r, C = x.size(0), self.r, self.GRAPH_CHUNK
        dec = self.decoder
        z = lambda n: torch.zeros(B, n, device=dev)  # noqa: E731
        enc = self.encoder(x, speaker_embedding)  # (eager: consumes the encoder's mask calls)
        enc_proj = self.encoder_proj(enc)
        # static inputs / carried state of the captured chunk
        st = [z(self.decoder_dims), z(self.lstm_dims), z(self.lstm_dims), z(self.lstm_dims),
              z(self.lstm_dims)]
        context = z(self.encoder_dims + self.speaker_embedding_size)
        prenet_in = z(self.n_mels)
        cum = torch.zeros(B, enc_proj.size(1), device=dev)
        d1, d2 = dec.prenet.fc1.out_features, dec.prenet.fc2.out_features
        stream = _dropout
        flat = torch.empty(C * B * (d1 + d2), device=dev)  # one copy per replay
        sizes = [B * d for _ in range(C) for d in (d1, d2)]
        masks = [v.view(B, -1) for v in torch.split(flat, sizes)]
        hist_m = torch.empty(C, B, self.n_mels, r, device=dev)
        hist_s = torch.empty(C, B, 1, enc_proj.size(1), device=dev)
        hist_stop = torch.empty(C, B, 1, device=dev)

        def chunk():
            state = tuple(st)
            ctx, pin = context, prenet_in
            dec.attn_net.cumulative = cum
            for i in range(C):
                mels, scores, state, ctx, stop = dec(enc, enc_proj, pin, state, ctx, 1, x, r)
                hist_m[i].copy_(mels)
                hist_s[i].copy_(scores)
                hist_stop[i].copy_(stop)
                pin = mels[:, :, -1]
            for a, b in zip(st, state):
                a.copy_(b)
            context.copy_(ctx)
            prenet_in.copy_(pin)
            cum.copy_(dec.attn_net.cumulative)

        def fill_masks(base):  # the stream's calls base.. of this chunk, in the eager order
            host = np.empty(flat.numel(), np.float32)
            o = 0
            for k, m in enumerate(masks):
                rng = np.random.Generator(np.random.PCG64([stream.seed, base + k]))
                keep = (rng.random(tuple(m.shape)) >= dec.prenet.p).astype(np.float32)
                host[o:o + m.numel()] = (keep / (1.0 - dec.prenet.p)).ravel()
                o += m.numel()
            flat.copy_(torch.from_numpy(host))

        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        saved = [t.clone() for t in st] + [context.clone(), prenet_in.clone(), cum.clone()]
        try:
            if stream is not None:
                _dropout = _StaticMasks(masks)
            with torch.cuda.stream(side):  # warm-up (allocations, library handles), then capture
                if stream is not None:
                    _dropout.i = 0
                chunk()
                if stream is not None:
                    _dropout.i = 0
                with torch.cuda.graph(g, stream=side):
                    chunk()
        finally:
            _dropout = stream
        torch.cuda.current_stream(dev).wait_stream(side)
        for t_, s_ in zip(st + [context, prenet_in, cum], saved):  # undo the warm-up chunk
            t_.copy_(s_)
        base = stream.calls if stream is not None else 0
        mel_outputs, attn = [], []
        done = 0
        for t0 in range(0, steps, C * r):
            if stream is not None:
                fill_masks(base + 2 * (t0 // r))
            g.replay()
            n = min(C, (steps - t0 + r - 1) // r)
            stops = (hist_stop[:n] > 0.5).all(dim=2).all(dim=1).cpu().numpy()
            ts = t0 + r * np.arange(n)
            hit = np.nonzero(stops & (ts > 10))[0]
            k = int(hit[0]) + 1 if len(hit) else n
            mel_outputs.extend(hist_m[i].clone() for i in range(k))
            attn.extend(hist_s[i].clone() for i in range(k))
            done += k
            if len(hit) or k < C:
                break
        if stream is not None:
            stream.calls = base + 2 * done
        mel_outputs = torch.cat(mel_outputs, dim=2)
        linear = self.post_proj(self.postnet(mel_outputs)).transpose(1, 2)
        return mel_outputs, linear, torch.cat(attn, 1)


def synth_tacotron_state_dict(model, seed=0):
    """Seeded stand-in weights for ``model``'s state dict (no checkpoint exists offline):
    xavier-uniform for matrices (the reference's init_model, tacotron.py:452-455), small
    uniform biases, randomised BatchNorm statistics. numpy PCG64, so any machine regenerates
    them bit for bit."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = {}
    for name, t in model.state_dict().items():
        shape = tuple(t.shape)
        leaf = name.rsplit('.', 1)[-1]
        if t.dtype != torch.float32:
            sd[name] = t.clone()
        elif leaf == 'running_mean':
            sd[name] = torch.from_numpy(rng.uniform(-0.1, 0.1, shape).astype(np.float32))
        elif leaf == 'running_var':
            sd[name] = torch.from_numpy(rng.uniform(0.5, 1.5, shape).astype(np.float32))
        elif 'bnorm' in name and leaf == 'weight':
            sd[name] = torch.from_numpy(rng.uniform(0.8, 1.2, shape).astype(np.float32))
        elif len(shape) >= 2:
            fan_in = int(np.prod(shape[1:]))
            fan_out = shape[0] * (int(np.prod(shape[2:])) if len(shape) > 2 else 1)
            b = float(np.sqrt(6.0 / (fan_in + fan_out)))
            sd[name] = torch.from_numpy(rng.uniform(-b, b, shape).astype(np.float32))
        elif name.endswith('stop_threshold'):
            sd[name] = t.clone()
        else:
            sd[name] = torch.from_numpy(rng.uniform(-0.05, 0.05, shape).astype(np.float32))
    return sd
