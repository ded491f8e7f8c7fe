"""GE2E speaker encoder (reference encoder/model.py:14-58): 3-layer LSTM over 40-channel mel
frames, ReLU(Linear) of the last layer's final hidden state, L2-normalised. State-dict names
match the reference (``lstm.*``, ``linear.*``, ``similarity_weight`` / ``similarity_bias``)."""
import numpy as np
import torch
from torch import nn

from .params import mel_n_channels, model_embedding_size, model_hidden_size, model_num_layers


class SpeakerEncoder(nn.Module):
    def __init__(self, device=None):
        super().__init__()
        self.lstm = nn.LSTM(input_size=mel_n_channels, hidden_size=model_hidden_size,
                            num_layers=model_num_layers, batch_first=True)
        self.linear = nn.Linear(model_hidden_size, model_embedding_size)
        self.relu = nn.ReLU()
        self.similarity_weight = nn.Parameter(torch.tensor([10.]))
        self.similarity_bias = nn.Parameter(torch.tensor([-5.]))
        if device is not None:
            self.to(device)

    def forward(self, utterances, hidden_init=None):
        """(B, n_frames, 40) -> (B, 768) unit-norm embeddings."""
        _, (hidden, _) = self.lstm(utterances, hidden_init)
        raw = self.relu(self.linear(hidden[-1]))
        return raw / torch.norm(raw, dim=1, keepdim=True)


def synth_encoder_state_dict(model, seed=0):
    """Seeded stand-in weights (torch-default-like uniform ranges; numpy PCG64)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    b = 1.0 / np.sqrt(model_hidden_size)
    sd = {}
    for name, t in model.state_dict().items():
        if name.startswith("similarity"):
            sd[name] = t.clone()
        else:
            sd[name] = torch.from_numpy(rng.uniform(-b, b, tuple(t.shape)).astype(np.float32))
    return sd
