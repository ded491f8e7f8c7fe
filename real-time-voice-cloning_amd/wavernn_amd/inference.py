"""Drop-in replacement of ``vocoder/inference.py`` (reference :1-101) on the MI355X.

Same module-level singleton and the same four functions:

* ``load_model(weights_fpath, voc_type='pytorch', verbose=True)``  (:11-53)
* ``is_loaded()``                                                   (:56-57)
* ``infer_waveform(mel, normalize=True, batched=True, target=None, overlap=None,
  progress_callback=None)``                                          (:59-95)
* ``set_seed(seed)``                                                (:97-101)

``voc_type`` 'pytorch' (the reference default) and 'mi355x' both select the GPU backend on a
checkpoint; 'libwavernn' loads a ``.bin`` file (vocoder/libwavernn/convert.py) into the
``wavernn_amd.libwavernn.Vocoder`` drop-in, as the reference does (:36-47, runtimeracer model).
Checkpoints are read with ``torch.load(..., weights_only=True)``.
"""
import os

import numpy as np

from . import base
from .hparams import sp

_model = None
_model_type = None
_device = 0
_seed = None


def load_model(weights_fpath, voc_type=base.VOC_TYPE_PYTORCH, verbose=True, device=None,
               state_dict=None, model_type=None):
    """Load a checkpoint ``{"model_state", "model_type"}`` (vocoder/train.py:308-324).

    ``state_dict``/``model_type`` may be given directly instead of a path (tests, bench).
    """
    global _model, _model_type, _device
    if voc_type not in (base.VOC_TYPE_PYTORCH, base.VOC_TYPE_MI355X, base.VOC_TYPE_CPP):
        raise NotImplementedError("Invalid vocoder of type '%s' provided. Aborting..." % voc_type)
    if device is None:
        device = int(os.environ.get('LOCAL_RANK', 0))
    _device = device
    if voc_type == base.VOC_TYPE_CPP:
        from .libwavernn import Vocoder
        # the reference hard-wires the runtimeracer topology here (vocoder/inference.py:38-39)
        _model = Vocoder(weights_fpath, model_type or base.MODEL_TYPE_RUNTIMERACER, verbose,
                         device=device)
        if _seed is not None:
            _model.setRandomSeed(_seed)
        _model.load()
        _model_type = voc_type
        if verbose:
            print("Loaded vocoder of model '%s' at path '%s'." % (_model_type, weights_fpath))
        return
    if state_dict is None:
        import torch
        checkpoint = torch.load(weights_fpath, map_location='cpu', weights_only=True)
        state_dict = checkpoint["model_state"]
        if model_type is None:
            model_type = checkpoint.get("model_type", base.MODEL_TYPE_FATCHORD)
    if model_type is None:
        model_type = base.MODEL_TYPE_FATCHORD
    try:
        model, _ = base.init_voc_model(model_type, device)
    except NotImplementedError as e:
        print(str(e))
        return
    model.load_state_dict(state_dict)
    if _seed is not None:
        model.set_seed(_seed)
    _model = model.eval()
    _model_type = model_type
    if verbose:
        print("Loaded vocoder of model '%s' at path '%s'." % (_model_type, weights_fpath))
        print("Model has been trained to step %d." % (_model.get_step()))


def is_loaded():
    return _model is not None


def infer_waveform(mel, normalize=True, batched=True, target=None, overlap=None,
                   progress_callback=None):
    """Infers the waveform of a mel spectrogram output by the synthesizer."""
    if _model is None or _model_type is None:
        raise Exception("Please load Wave-RNN in memory before using it")
    if _model_type == base.VOC_TYPE_CPP:
        return _model.vocode_mel(mel=mel, normalize=normalize, progress_callback=progress_callback)
    hp_wavernn = base.hparams_for(_model_type)
    if target is None:
        target = hp_wavernn.gen_target
    if overlap is None:
        overlap = hp_wavernn.gen_overlap
    if normalize:
        mel = mel / sp.max_abs_value
    mel = np.asarray(mel, dtype=np.float32)[None, ...]
    wav = _model.generate(mel, batched, target, overlap, hp_wavernn.mu_law, sp.preemphasize,
                          progress_callback)
    return wav


def set_seed(seed):
    global _seed
    _seed = seed
    if _model is not None:
        if _model_type == base.VOC_TYPE_CPP:
            _model.setRandomSeed(seed)
        else:
            _model.set_seed(seed)


def get_model():
    return _model
