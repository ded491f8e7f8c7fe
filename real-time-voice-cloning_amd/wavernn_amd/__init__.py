"""MI355X-native WaveRNN vocoder inference (drop-in for the reference's vocoder path).

Public surface mirrors the reference (RuntimeRacer/Real-Time-Voice-Cloning):
``wavernn_amd.inference`` == ``vocoder.inference``; ``wavernn_amd.base`` == ``vocoder.models.base``;
``wavernn_amd.model.WaveRNN`` == ``vocoder.models.{fatchord,runtimeracer}_version.WaveRNN``.
"""
__version__ = '0.1.0'
