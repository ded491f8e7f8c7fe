"""Speaker encoder side of the end-to-end path: GE2E LSTM encoder on
PyTorch-ROCm; drop-in for the reference's ``encoder`` package names used by ``demo_cli.py``."""
