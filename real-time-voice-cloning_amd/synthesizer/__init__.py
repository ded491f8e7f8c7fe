"""Synthesizer side of the end-to-end path: Tacotron on PyTorch-ROCm feeding
the MI355X vocoder. Drop-in for the reference's ``synthesizer`` package names used by
``demo_cli.py`` / the toolbox (``synthesizer.inference.Synthesizer``)."""
