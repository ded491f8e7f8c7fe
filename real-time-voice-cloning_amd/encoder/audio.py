"""Waveform preprocessing and mel features of the speaker encoder.

Follows the reference's ``encoder/audio.py`` (``preprocess_wav`` :16-51, ``wav_to_mel_spectrogram``
:54-66, ``trim_long_silences`` :73-117, ``normalize_volume`` :120-126). Its third-party steps
are absent from this image and restated: ``librosa.feature.melspectrogram`` (power-2 STFT with
a periodic Hann window, ``center=True`` constant padding, Slaney mel filterbank with Slaney
area normalisation -- librosa's defaults) in numpy, ``librosa.resample`` by
``scipy.signal.resample_poly``, and ``webrtcvad`` (VAD silence trimming) is skipped with a
warning when the package is missing (the reference would fail). These restatements are
"parity unpinned" (librosa is not importable here); the model itself is pinned
(tests/golden/e2e_*.npz).
"""
from math import gcd
from warnings import warn

import numpy as np

from .params import (audio_norm_target_dBFS, mel_n_channels, mel_window_length, mel_window_step,
                     sampling_rate, vad_max_silence_length, vad_moving_average_width,
                     vad_window_length)

try:
    import webrtcvad
except ImportError:
    webrtcvad = None

int16_max = (2 ** 15) - 1


def _hz_to_mel(f):
    """Slaney mel scale (librosa htk=False): linear below 1 kHz, log above."""
    f = np.asarray(f, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-10) / min_log_hz) / logstep,
                    f / f_sp)


def _mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def mel_filterbank(sr, n_fft, n_mels, fmin=0.0, fmax=None):
    """(n_mels, 1 + n_fft // 2) triangular filters, Slaney-normalised (librosa.filters.mel)."""
    fmax = sr / 2.0 if fmax is None else fmax
    fft_freqs = np.linspace(0, sr / 2.0, 1 + n_fft // 2)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fft_freqs[None, :]
    weights = np.maximum(0, np.minimum(-ramps[:-2] / fdiff[:-1, None], ramps[2:] / fdiff[1:, None]))
    weights *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return weights.astype(np.float32)


def power_stft(wav, n_fft, hop):
    """|STFT|^2 with a periodic Hann window, centred frames (zero padding), (1 + n_fft/2, T)."""
    y = np.pad(np.asarray(wav, dtype=np.float32), n_fft // 2, mode="constant")
    n_frames = 1 + (len(y) - n_fft) // hop
    win = (0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n_fft) / n_fft)).astype(np.float32)
    idx = np.arange(n_fft)[None, :] + hop * np.arange(n_frames)[:, None]
    spec = np.fft.rfft(y[idx] * win[None, :], axis=1)
    return (np.abs(spec) ** 2).T


def wav_to_mel_spectrogram(wav):
    """(T, 40) float32 mel power frames (not log) of a preprocessed waveform."""
    n_fft = int(sampling_rate * mel_window_length / 1000)
    hop = int(sampling_rate * mel_window_step / 1000)
    S = power_stft(wav, n_fft, hop)
    frames = mel_filterbank(sampling_rate, n_fft, mel_n_channels).astype(np.float64) @ S
    return frames.astype(np.float32).T


def normalize_volume(wav, target_dBFS, increase_only=False, decrease_only=False):
    if increase_only and decrease_only:
        raise ValueError("Both increase only and decrease only are set")
    dBFS_change = target_dBFS - 10 * np.log10(np.mean(wav ** 2))
    if (dBFS_change < 0 and increase_only) or (dBFS_change > 0 and decrease_only):
        return wav
    return wav * (10 ** (dBFS_change / 20))


def trim_long_silences(wav):
    """VAD-based removal of long silences (audio.py:73-117); identity without webrtcvad."""
    if webrtcvad is None:
        warn("webrtcvad is unavailable: long silences are not trimmed")
        return wav
    import struct
    from scipy.ndimage import binary_dilation
    spw = (vad_window_length * sampling_rate) // 1000
    wav = wav[:len(wav) - (len(wav) % spw)]
    pcm = struct.pack("%dh" % len(wav), *(np.round(wav * int16_max)).astype(np.int16))
    vad = webrtcvad.Vad(mode=3)
    flags = np.array([vad.is_speech(pcm[s * 2:(s + spw) * 2], sample_rate=sampling_rate)
                      for s in range(0, len(wav), spw)])
    w = vad_moving_average_width
    padded = np.concatenate((np.zeros((w - 1) // 2), flags, np.zeros(w // 2)))
    ret = np.cumsum(padded, dtype=float)
    ret[w:] = ret[w:] - ret[:-w]
    mask = np.round(ret[w - 1:] / w).astype(bool)
    mask = binary_dilation(mask, np.ones(vad_max_silence_length + 1))
    return wav[np.repeat(mask, spw)]


def preprocess_wav(fpath_or_wav, source_sr=None, normalize=True, trim_silence=True):
    """Resample to 16 kHz, normalise the volume to -30 dBFS (increase only), trim silences."""
    if isinstance(fpath_or_wav, (str, bytes)) or hasattr(fpath_or_wav, "__fspath__"):
        from scipy.io import wavfile
        source_sr, wav = wavfile.read(fpath_or_wav)
        wav = wav.astype(np.float32) / (np.iinfo(wav.dtype).max if wav.dtype.kind == "i" else 1.0)
        if wav.ndim > 1:
            wav = wav.mean(axis=1)
    else:
        wav = fpath_or_wav
    if source_sr is not None and source_sr != sampling_rate:
        from scipy.signal import resample_poly
        g = gcd(int(source_sr), sampling_rate)
        wav = resample_poly(wav, sampling_rate // g, int(source_sr) // g).astype(np.float32)
    if normalize:
        wav = normalize_volume(wav, audio_norm_target_dBFS, increase_only=True)
    if trim_silence:
        wav = trim_long_silences(wav)
    return wav
