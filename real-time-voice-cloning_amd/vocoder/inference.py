"""``vocoder.inference`` drop-in: re-exports wavernn_amd.inference (reference vocoder/inference.py)."""
from wavernn_amd.inference import (load_model, is_loaded, infer_waveform, set_seed,  # noqa: F401
                                   get_model)
