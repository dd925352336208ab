"""Audio input. The reference decodes files with pydub/ffmpeg (nano_audio.py:3-30), absent here: this
loader reads PCM WAV (stdlib `wave`) or .npy, downmixes to mono, normalises ints by 2^(bits-1) like the
reference, and resamples linearly to 16 kHz when needed. numpy arrays pass straight through."""
import wave

import numpy as np


def load_audio(audio, sample_rate=16000, start_second=None, duration=None):
    if isinstance(audio, np.ndarray):
        x = audio.astype(np.float32)
        sr = sample_rate
    elif str(audio).endswith(".npy"):
        x = np.load(audio, allow_pickle=False).astype(np.float32)
        sr = sample_rate
    else:
        with wave.open(str(audio), "rb") as w:
            sr, ch, sw, n = w.getframerate(), w.getnchannels(), w.getsampwidth(), w.getnframes()
            raw = w.readframes(n)
        dt = {1: np.uint8, 2: np.int16, 4: np.int32}[sw]
        x = np.frombuffer(raw, dt).astype(np.float64)
        if sw == 1:
            x -= 128.0
        x = x.reshape(-1, ch).mean(1) / float(1 << (8 * sw - 1))
        x = x.astype(np.float32)
    if sr != sample_rate and x.size:
        t = np.arange(int(round(x.size * sample_rate / sr))) * (sr / sample_rate)
        x = np.interp(t, np.arange(x.size), x).astype(np.float32)
    if start_second:
        x = x[int(start_second * sample_rate):]
    if duration:
        x = x[:int(duration * sample_rate)]
    return x
