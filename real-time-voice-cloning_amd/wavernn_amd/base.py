"""Model-type registry and factory (vocoder/models/base.py:8-120 of the reference).

``VOC_TYPE_MI355X`` is the backend added by this package; ``VOC_TYPE_PYTORCH`` is accepted as
an alias so unmodified callers of ``load_model(path)`` land on the GPU path; ``VOC_TYPE_CPP``
('libwavernn') loads ``.bin`` files (wavernn_amd/libwavernn.py). All three registered model
types are built: fatchord, runtimeracer and geneing (modes BITS and MOL; its Beta 'RAW' mode
raises NotImplementedError).
"""
import numpy as np

from .hparams import sp, wavernn_fatchord, wavernn_geneing, wavernn_runtimeracer
from .model import WaveRNN, MODEL_TYPE_FATCHORD, MODEL_TYPE_GENEING, MODEL_TYPE_RUNTIMERACER

VOC_TYPE_CPP = 'libwavernn'
VOC_TYPE_PYTORCH = 'pytorch'
VOC_TYPE_MI355X = 'mi355x'


def hparams_for(model_type):
    if model_type == MODEL_TYPE_FATCHORD:
        return wavernn_fatchord
    if model_type == MODEL_TYPE_RUNTIMERACER:
        return wavernn_runtimeracer
    if model_type == MODEL_TYPE_GENEING:
        return wavernn_geneing
    raise NotImplementedError("Invalid model of type '%s' provided. Aborting..." % model_type)


def init_voc_model(model_type, device, override_hp_fatchord=None, override_hp_geneing=None,
                   override_hp_runtimeracer=None):
    """base.py:18-109: build the model for a type; returns (model, pruner=None)."""
    if model_type == MODEL_TYPE_FATCHORD:
        hparams = override_hp_fatchord or wavernn_fatchord
    elif model_type == MODEL_TYPE_RUNTIMERACER:
        hparams = override_hp_runtimeracer or wavernn_runtimeracer
    elif model_type == MODEL_TYPE_GENEING:
        hparams = override_hp_geneing or wavernn_geneing
    else:
        raise NotImplementedError("Invalid model of type '%s' provided. Aborting..." % model_type)
    assert np.cumprod(hparams.upsample_factors)[-1] == sp.hop_size
    dev = 0
    if isinstance(device, int):
        dev = device
    elif hasattr(device, 'index') and device.index is not None:
        dev = device.index
    model = WaveRNN(
        rnn_dims=hparams.rnn_dims,
        fc_dims=hparams.fc_dims,
        bits=hparams.bits,
        pad=hparams.pad,
        upsample_factors=hparams.upsample_factors,
        feat_dims=sp.num_mels,
        compute_dims=hparams.compute_dims,
        res_out_dims=hparams.res_out_dims,
        res_blocks=hparams.res_blocks,
        hop_length=sp.hop_size,
        sample_rate=sp.sample_rate,
        mode=hparams.mode,
        model_type=model_type,
        device=dev,
    )
    return model, None


def get_model_type(model):
    if isinstance(model, WaveRNN):
        return model.model_type
    raise NotImplementedError("Provided object is not a valid vocoder model.")
