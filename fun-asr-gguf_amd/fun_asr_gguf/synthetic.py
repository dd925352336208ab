"""Seeded synthetic 16 kHz input for tests and benchmarks.

Real recordings (input.mp3 needs ffmpeg, vad_example.wav is absent) cannot be decoded in this image,
so every clip is: 3 harmonic linear chirps (fundamental 100 -> 1000 Hz, harmonics x1..x3, amplitude 0.2)
plus white noise sigma 0.01, rng = np.random.default_rng(1000 + clip_idx), clipped to [-1, 1).
"""
import numpy as np

SAMPLE_RATE = 16000


def synth_audio(n_samples: int, clip_idx: int = 0) -> np.ndarray:
    rng = np.random.default_rng(1000 + clip_idx)
    t = np.arange(n_samples, dtype=np.float64) / SAMPLE_RATE
    dur = max(n_samples / SAMPLE_RATE, 1e-3)
    f0 = 100.0 + 50.0 * rng.random()
    f1 = 1000.0 - 100.0 * rng.random()
    phase = 2 * np.pi * (f0 * t + (f1 - f0) * t * t / (2 * dur))
    x = np.zeros(n_samples, dtype=np.float64)
    for h in (1, 2, 3):
        x += 0.2 * np.sin(h * phase + rng.random() * 2 * np.pi)
    x += rng.normal(0.0, 0.01, n_samples)
    return np.clip(x, -1.0, 1.0 - 2.0 ** -15).astype(np.float32)
