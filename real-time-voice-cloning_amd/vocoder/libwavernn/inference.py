"""``vocoder.libwavernn.inference`` drop-in: re-exports wavernn_amd.libwavernn.Vocoder."""
from wavernn_amd.libwavernn import Vocoder  # noqa: F401
