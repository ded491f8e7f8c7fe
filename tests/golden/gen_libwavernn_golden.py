"""Golden fixtures of the reference's libwavernn host path (survey container only).

Imports ``vocoder/libwavernn/inference.py`` of the reference from /root/reference with the
import shims of gen_golden.py (its ``WaveRNNVocoder`` extension is unbuildable here, so a stub
module stands in for the import only) and records, on seeded synthetic inputs:

* ``fold_mel_with_overlap`` (inference.py:131-162) -- the raw-mel folding;
* ``unfold_wav_with_overlap`` (inference.py:164-195) -- the chunk cross-fade;
* the whole ``Vocoder.vocode_mel`` (inference.py:60-128) with N processing wrappers whose
  ``melToWav`` is replaced by a deterministic function of the chunk (``fake_mel_to_wav`` below,
  also used by the test), so every host-side step -- target choice, folding, unfold, mu-law
  decode, de-emphasis, fade-out -- is pinned against the reference's own code.

Usage:  python tests/golden/gen_libwavernn_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden  # noqa: E402  (shims, REPO path setup)

CASES = {
    # name: (model_type, n_frames, n_wrappers, mel_seed)
    'rr_t120_w6': ('runtimeracer-wavernn', 120, 6, 31),
    'rr_t57_w4': ('runtimeracer-wavernn', 57, 4, 32),
    'rr_t40_w1': ('runtimeracer-wavernn', 40, 1, 33),
    'fc_t90_w5': ('fatchord-wavernn', 90, 5, 34),
}


def fake_mel_to_wav(chunk, hop=200):
    """Deterministic stand-in for WaveRNNVocoder.melToWav: float32 samples in [-1, 1]."""
    chunk = np.asarray(chunk, dtype=np.float32)
    L = chunk.shape[1] * hop
    phase = float(np.sum(chunk, dtype=np.float64))
    return (0.9 * np.sin(np.arange(L, dtype=np.float64) * 0.013 + phase)).astype(np.float32)


class FakeWrapper:
    def melToWav(self, chunk):
        return fake_mel_to_wav(chunk)


def main():
    gen_golden.install_shims()
    from vocoder.libwavernn import inference as ref  # noqa: E402
    out = {}
    for name, (mt, T, nw, seed) in CASES.items():
        rng = np.random.default_rng(seed)
        mel = rng.uniform(-4, 4, (80, T)).astype(np.float32)
        v = ref.Vocoder('unused.bin', mt, verbose=False)
        v._processing_thread_wrappers = [FakeWrapper() for _ in range(nw)]
        wav = v.vocode_mel(mel.copy(), normalize=True)
        folded = v.fold_mel_with_overlap(mel / 4.0, 2750, 1000)
        fw = rng.uniform(-1, 1, (5, 3000)).astype(np.float32)
        unf = v.unfold_wav_with_overlap(fw.copy(), 1000, 500)
        np.savez_compressed(os.path.join(HERE, f'libwavernn_{name}.npz'), mel=mel, wav=wav,
                            folded=np.stack(folded), fw=fw, unfolded=unf,
                            meta=np.array([T, nw, seed]), model_type=np.array(mt))
        out[name] = (wav.shape, len(folded), unf.shape)
        print(name, out[name])


if __name__ == '__main__':
    main()
