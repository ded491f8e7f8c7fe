"""Drop-in for the reference's ``encoder/inference.py``: ``load_model`` (:16-37), ``is_loaded``
(:40-41), ``embed_frames_batch`` (:44-57), ``compute_partial_slices`` (:60-112),
``embed_utterance`` (:115-156) and the re-exported ``preprocess_wav``. The LSTM runs on
PyTorch-ROCm; outputs are numpy on the host, as in the reference."""
import numpy as np
import torch

from . import audio
from .audio import preprocess_wav  # noqa: F401
from .model import SpeakerEncoder, synth_encoder_state_dict
from .params import mel_window_step, partials_n_frames, sampling_rate

_model = None  # type: SpeakerEncoder
_device = None


def load_model(weights_fpath=None, device=None, use_tqdm=False, state_dict=None,
               random_weights=None):
    """Checkpoint (``torch.load(weights_only=True)``) or, offline, a given / seeded state dict."""
    global _model, _device
    _device = torch.device(device) if device is not None else \
        torch.device("cuda" if torch.cuda.is_available() else "cpu")
    _model = SpeakerEncoder(_device)
    if state_dict is None and random_weights is not None:
        state_dict = synth_encoder_state_dict(_model, random_weights)
    step = 0
    if state_dict is None:
        ckpt = torch.load(weights_fpath, map_location=_device, weights_only=True)
        state_dict, step = ckpt["model_state"], ckpt.get("step", 0)
    _model.load_state_dict(state_dict)
    _model.eval()
    print("Loaded encoder \"%s\" trained to step %d" % (weights_fpath, step))


def is_loaded():
    return _model is not None


def embed_frames_batch(frames_batch):
    if _model is None:
        raise Exception("Model was not loaded. Call load_model() before inference.")
    frames = torch.from_numpy(frames_batch).to(_device)
    with torch.no_grad():
        return _model.forward(frames).detach().cpu().numpy()


def compute_partial_slices(n_samples, partial_utterance_n_frames=partials_n_frames,
                           min_pad_coverage=0.75, overlap=0.5):
    assert 0 <= overlap < 1
    assert 0 < min_pad_coverage <= 1
    spf = int((sampling_rate * mel_window_step / 1000))
    n_frames = int(np.ceil((n_samples + 1) / spf))
    step = max(int(np.round(partial_utterance_n_frames * (1 - overlap))), 1)
    wav_slices, mel_slices = [], []
    for i in range(0, max(1, n_frames - partial_utterance_n_frames + step + 1), step):
        mel_slices.append(slice(i, i + partial_utterance_n_frames))
        wav_slices.append(slice(i * spf, (i + partial_utterance_n_frames) * spf))
    last = wav_slices[-1]
    coverage = (n_samples - last.start) / (last.stop - last.start)
    if coverage < min_pad_coverage and len(mel_slices) > 1:
        mel_slices, wav_slices = mel_slices[:-1], wav_slices[:-1]
    return wav_slices, mel_slices


def embed_utterance(wav, using_partials=True, return_partials=False, **kwargs):
    if not using_partials:
        embed = embed_frames_batch(audio.wav_to_mel_spectrogram(wav)[None, ...])[0]
        return (embed, None, None) if return_partials else embed
    wave_slices, mel_slices = compute_partial_slices(len(wav), **kwargs)
    max_len = wave_slices[-1].stop
    if max_len >= len(wav):
        wav = np.pad(wav, (0, max_len - len(wav)), "constant")
    frames = audio.wav_to_mel_spectrogram(wav)
    partial_embeds = embed_frames_batch(np.array([frames[s] for s in mel_slices]))
    raw = np.mean(partial_embeds, axis=0)
    embed = raw / np.linalg.norm(raw, 2)
    return (embed, partial_embeds, wave_slices) if return_partials else embed
