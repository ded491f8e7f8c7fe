"""``vocoder.libwavernn.convert`` drop-in: checkpoint -> libwavernn .bin (wavernn_amd.convert)."""
from wavernn_amd.convert import convert_model, compress, write_bin  # noqa: F401
