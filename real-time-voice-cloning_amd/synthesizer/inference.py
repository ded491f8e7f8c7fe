"""Drop-in for the reference's ``synthesizer/inference.py`` (Tacotron path).

Same class and module API as the reference (``Synthesizer`` :13-163 with ``load``,
``is_loaded``, ``get_model_type``, ``synthesize_spectrograms``; module-level ``load_model``,
``is_loaded``, ``synthesize_spectrograms`` :166-198; ``pad1d`` :234) on PyTorch-ROCm.
Checkpoints load with ``torch.load(..., weights_only=True)``. ``state_dict=`` (or
``random_weights=seed``) stands in for a checkpoint file where none is available offline.

The ForwardTacotron / FastPitch model types of the reference are out of scope; the
Griffin-Lim / librosa audio helpers are not part of the vocoder path.
"""
from pathlib import Path
from typing import List, Union

import numpy as np
import torch

from .hparams import preprocessing, sp, sv2tts, tacotron as hp_tacotron
from .tacotron import Tacotron, synth_tacotron_state_dict
from .text import symbols, text_to_sequence

MODEL_TYPE_TACOTRON = 'tacotron'


def build_tacotron(device, hp=None):
    """synthesizer/models/base.py:13-37 for the Tacotron type."""
    hp = hp or hp_tacotron
    return Tacotron(embed_dims=hp.embed_dims, num_chars=len(symbols), encoder_dims=hp.encoder_dims,
                    decoder_dims=hp.decoder_dims, n_mels=sp.num_mels, fft_bins=sp.num_mels,
                    postnet_dims=hp.postnet_dims, encoder_K=hp.encoder_K, lstm_dims=hp.lstm_dims,
                    postnet_K=hp.postnet_K, num_highways=hp.num_highways, dropout=hp.dropout,
                    stop_threshold=hp.stop_threshold,
                    speaker_embedding_size=sv2tts.speaker_embedding_size).to(device)


def pad1d(x, max_len, pad_value=0):
    return np.pad(x, (0, max_len - len(x)), mode="constant", constant_values=pad_value)


class Synthesizer:

    def __init__(self, model_fpath: Path = None, verbose=True, device=None, state_dict=None,
                 random_weights=None):
        self.model_fpath = model_fpath
        self.verbose = verbose
        if device is None:
            device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.device = torch.device(device)
        self._state_dict = state_dict
        self._random_weights = random_weights
        self._model = None
        self._model_type = None
        if verbose:
            print("Synthesizer using device:", self.device)

    def is_loaded(self):
        return self._model is not None

    def get_model_type(self):
        if not self.is_loaded():
            self.load()
        return self._model_type

    def load(self):
        model = build_tacotron(self.device)
        if self._state_dict is not None:
            model.load_state_dict(self._state_dict)
        elif self._random_weights is not None:
            model.load_state_dict(synth_tacotron_state_dict(model, self._random_weights))
        else:
            ckpt = torch.load(str(self.model_fpath), map_location=self.device, weights_only=True)
            mt = ckpt.get("model_type", MODEL_TYPE_TACOTRON)
            if mt != MODEL_TYPE_TACOTRON:
                raise NotImplementedError("Synthesizer model type '%s' is not supported "
                                          "(Tacotron only)" % mt)
            model.load(self.model_fpath, checkpoint=ckpt)
        model.eval()
        self._model = model
        self._model_type = MODEL_TYPE_TACOTRON
        if self.verbose:
            print("Loaded synthesizer of model '%s'; trained to step %d." % (self._model_type,
                                                                              model.get_step()))

    def synthesize_spectrograms(self, texts: List[str],
                                embeddings: Union[np.ndarray, List[np.ndarray]],
                                return_alignments=False, steps=2000):
        """inference.py:79-164: texts + speaker embeddings -> list of (80, Mi) mels."""
        if not self.is_loaded():
            self.load()
        inputs = [text_to_sequence(t.strip(), preprocessing.cleaner_names) for t in texts]
        if not isinstance(embeddings, list):
            embeddings = [embeddings]
        bs = preprocessing.synthesis_batch_size
        specs, alignments = [], None
        for i in range(0, len(inputs), bs):
            batch = inputs[i:i + bs]
            max_len = max(len(t) for t in batch)
            chars = torch.tensor(np.stack([pad1d(t, max_len) for t in batch])).long().to(self.device)
            spk = torch.tensor(np.stack(embeddings[i:i + bs])).float().to(self.device)
            _, mels, alignments = self._model.generate(chars, spk, steps=steps)
            for m in mels.detach().cpu().numpy():
                while m.shape[1] > 1 and np.max(m[:, -1]) < hp_tacotron.stop_threshold:  # silent tail
                    m = m[:, :-1]
                specs.append(m)
        return (specs, alignments) if return_alignments else specs


_model = None  # type: Synthesizer


def load_model(weights_fpath, verbose=True, **kw):
    global _model
    _model = Synthesizer(weights_fpath, verbose, **kw)
    _model.load()


def is_loaded():
    return _model is not None and _model.is_loaded()


def get_model_type():
    if not is_loaded():
        raise Exception("Please load Synthesizer in memory before using it")
    return _model.get_model_type()


def synthesize_spectrograms(texts, embeddings, return_alignments=False, **kw):
    if not is_loaded():
        raise Exception("Please load Synthesizer in memory before using it")
    return _model.synthesize_spectrograms(texts, embeddings, return_alignments, **kw)
