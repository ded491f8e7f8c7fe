"""Synthesizer-side fields of the reference's config/hparams.py (:33-35 sv2tts, :52-95
preprocessing, :97-141 tacotron) -- inference fields only."""
from wavernn_amd.hparams import HParams, sp  # noqa: F401  (sp: signal processing, shared)

sv2tts = HParams(speaker_embedding_size=768)

preprocessing = HParams(
    max_mel_frames=1200,
    rescale=True,
    rescaling_max=0.9,
    synthesis_batch_size=24,
    cleaner_names=["english_cleaners"],
)

tacotron = HParams(
    embed_dims=256,
    encoder_dims=128,
    decoder_dims=256,
    postnet_dims=128,
    encoder_K=16,
    lstm_dims=512,
    postnet_K=8,
    num_highways=4,
    dropout=0.5,
    stop_threshold=-3.4,
)
