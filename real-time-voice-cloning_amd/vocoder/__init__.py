"""Drop-in package name of the reference: put ``real-time-voice-cloning_amd`` on sys.path and
``from vocoder import inference as vocoder`` (demo_cli.py:11 of the reference) resolves to the
MI355X backend."""
