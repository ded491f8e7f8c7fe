"""encoder/params_data.py and encoder/params_model.py of the reference (inference fields)."""
mel_window_length = 25  # ms
mel_window_step = 10    # ms
mel_n_channels = 40
sampling_rate = 16000
partials_n_frames = 160
inference_n_frames = 80
vad_window_length = 30  # ms
vad_moving_average_width = 8
vad_max_silence_length = 6
audio_norm_target_dBFS = -30
model_hidden_size = 768
model_embedding_size = 768
model_num_layers = 3
