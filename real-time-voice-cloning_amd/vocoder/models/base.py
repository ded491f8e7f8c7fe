"""``vocoder.models.base`` drop-in (reference vocoder/models/base.py)."""
from wavernn_amd.base import (VOC_TYPE_CPP, VOC_TYPE_PYTORCH, VOC_TYPE_MI355X,  # noqa: F401
                              MODEL_TYPE_FATCHORD, MODEL_TYPE_GENEING, MODEL_TYPE_RUNTIMERACER,
                              init_voc_model, get_model_type)
