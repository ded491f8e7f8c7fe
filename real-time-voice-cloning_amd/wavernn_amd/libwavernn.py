"""Drop-in for the reference's libwavernn backend (``vocoder/libwavernn/inference.py``).

The reference's ``voc_type='libwavernn'`` path loads a ``.bin`` weight file (convert.py) into
one C++ ``WaveRNNVocoder.Vocoder`` per physical CPU core, folds the RAW mel into as many chunks
as there are cores (inference.py:96-108), vocodes every chunk as an independent *unbatched*
sequence on its own thread (``melToWav``, net_impl.cpp:154-224) and cross-fades the chunks back
together on the host (inference.py:164-195) before mu-law decoding, de-emphasis and the fade-out.

Here the chunks are the fold rows of ONE unbatched multi-utterance call on the MI355X (every
chunk has the same length, so they run side by side in the persistent recurrence), the weights
come from the same ``.bin`` file through the C-ABI reader (``wrnn_load_bin``), and the host steps
are the reference's own numpy arithmetic. ``max_threads`` plays the role of the core count: the
number of chunks the mel is split into (default: the rows of one persistent launch, 24).

Sampling follows this build's noise contract (DESIGN.md "RNG contract"), not the C++ library's
``std::`` random engine (net_impl.cpp:128-143), which cannot be reproduced here; everything
else is pinned by ``tests/golden/libwavernn_*.npz`` (generated from the reference's code).
"""
import math

import numpy as np

from . import base
from .audio import decode_mu_law, de_emphasis
from .hparams import sp

DEFAULT_CHUNKS = 24


class Vocoder:

    def __init__(self, model_fpath, model_type, verbose=True, device=0):
        self.model_fpath = model_fpath
        self.model_type = model_type
        self.verbose = verbose
        self.device = device
        self._model = None
        self._n_chunks = 0
        self._seed = None
        if verbose:
            print("Instantiated MI355X WaveRNN vocoder wrapper for model: ", self.model_fpath)

    # inference.py:35-50 -- one model on the GPU; max_threads = chunk count
    def load(self, max_threads=None):
        hp = base.hparams_for(self.model_type)
        if hp.mode != 'RAW':
            raise NotImplementedError("libwavernn vocodes RAW (categorical) models only")
        model, _ = base.init_voc_model(self.model_type, self.device)
        model.load_bin(self.model_fpath)
        if self._seed is not None:
            model.set_seed(self._seed)
        self._model = model
        self._n_chunks = int(max_threads) if max_threads else DEFAULT_CHUNKS

    @property
    def _processing_thread_wrappers(self):
        # the reference's readiness check (inference.py:80-83) counts wrappers
        return [self._model] * self._n_chunks if self._model is not None else []

    def vocode_mel(self, mel, normalize=True, progress_callback=None):
        """inference.py:52-128."""
        hp_wavernn = base.hparams_for(self.model_type)
        if normalize:
            mel = mel / sp.max_abs_value
        wave_len = mel.shape[1] * sp.hop_size
        wrapper_count = len(self._processing_thread_wrappers)
        if wrapper_count == 0:
            raise RuntimeError("No processing thread wrappers. Did you properly load the Vocoder "
                               "instance? Aborting...")
        elif wrapper_count == 1:
            output = self._vocode_chunks([mel], progress_callback)[0]
        else:
            min_target = hp_wavernn.gen_target
            min_overlap = hp_wavernn.gen_overlap
            optimal_target = math.ceil(((wave_len - min_overlap) / wrapper_count) - min_overlap)
            if optimal_target < min_target:
                optimal_target = min_target
            mels = self.fold_mel_with_overlap(mel, optimal_target, min_overlap)
            output = np.stack(self._vocode_chunks(mels, progress_callback), axis=0)
            output = self.unfold_wav_with_overlap(output, optimal_target, min_overlap)
        if hp_wavernn.mu_law:
            output = decode_mu_law(output, 2 ** hp_wavernn.bits, False)
        if sp.preemphasize:
            output = de_emphasis(output)
        fade_out = np.linspace(1, 0, 20 * sp.hop_size)
        output = output[:wave_len]
        output[-20 * sp.hop_size:] *= fade_out
        return output

    def _vocode_chunks(self, chunks, progress_callback=None):
        """melToWav of every chunk: one unbatched call, one fold row per chunk; float32 samples
        ``(2 k) / (n - 1) - 1`` computed in double and stored as float (net_impl.cpp:219-221)."""
        import torch
        m = self._model
        dev = torch.device('cuda', m.device)
        mels = [torch.from_numpy(np.ascontiguousarray(c, dtype=np.float32)).to(dev) for c in chunks]
        out, roff, S = m.generate_batch_device(mels, False, 0, 0, progress_callback)
        labels = out.cpu().numpy()
        n = m.n_classes
        return [((2. * labels[roff[u]].astype(np.float64)) / (n - 1.) - 1.).astype(np.float32)
                for u in range(len(chunks))]

    def vocode_thread(self, tID, chunk):
        return self._vocode_chunks([chunk])[0]

    def fold_mel_with_overlap(self, mel, target, overlap):
        """inference.py:131-162: folding of the raw mel (before upsampling)."""
        mel_len = mel.shape[1]
        mel_target = math.ceil(target / sp.hop_size)
        mel_overlap = math.ceil(overlap / sp.hop_size)
        num_folds = (mel_len - mel_overlap) // (mel_target + mel_overlap)
        extended_len = num_folds * (mel_overlap + mel_target) + mel_overlap
        remaining = mel_len - extended_len
        if remaining != 0:
            num_folds += 1
            padding = mel_target + 2 * mel_overlap - remaining
            padded_mel = np.zeros(shape=(mel.shape[0], mel_len + padding), dtype=np.float32)
            padded_mel[:, :mel_len] = mel
            mel = padded_mel
        span = mel_target + 2 * mel_overlap
        step = mel_target + mel_overlap
        return [mel[:, i * step:i * step + span] for i in range(num_folds)]

    def unfold_wav_with_overlap(self, wav, target, overlap):
        """inference.py:164-195: equal-power cross-fade of the chunk outputs."""
        num_folds, length = wav.shape
        target = length - 2 * overlap
        total_len = num_folds * (target + overlap) + overlap
        silence_len = overlap // 2
        fade_len = overlap - silence_len
        silence = np.zeros((silence_len), dtype=np.float64)
        t = np.linspace(-1, 1, fade_len, dtype=np.float64)
        fade_in = np.concatenate([silence, np.sqrt(0.5 * (1 + t))])
        fade_out = np.concatenate([np.sqrt(0.5 * (1 - t)), silence])
        wav[:, :overlap] *= fade_in
        wav[:, -overlap:] *= fade_out
        unfolded = np.zeros((total_len), dtype=np.float64)
        for i in range(num_folds):
            start = i * (target + overlap)
            unfolded[start:start + target + 2 * overlap] += wav[i]
        return unfolded

    def setRandomSeed(self, seed):
        self._seed = seed
        if self._model is not None:
            self._model.set_seed(seed)
