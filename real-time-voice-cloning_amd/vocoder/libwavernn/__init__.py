"""``vocoder.libwavernn`` drop-in (reference vocoder/libwavernn/): .bin weights on the MI355X."""
