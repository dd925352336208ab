"""F1-F4 frontend restatement (numpy) — TEST INFRASTRUCTURE ONLY.

Follows EncoderExportWrapperPaddable.forward, /root/reference/fun_asr_gguf/model_definition.py:269-311,
STFT_Process (:244-256), SinusoidalPositionEncoder (:9-28) and the HTK mel filterbank built in
01-Export-Encoder-Adaptor-CTC.py:102 with torchaudio.functional.melscale_fbanks(201, 20, 8000, 80,
16000, None, 'htk'). torchaudio is absent from this image (third-party, unpinned in
requirements.txt); its published algorithm is restated in `mel_fbank()` below.
"""
import math
import numpy as np

SR = 16000
N_FFT = 400
HOP = 160
N_FREQ = N_FFT // 2 + 1  # 201
N_MELS = 80
PRE_EMPH = 0.97
LFR_M, LFR_N = 7, 6


def _linspace_f32(start, end, steps):
    # torch CPU linspace (RangeFactoriesKernel.cpp): f32 step, two-sided evaluation.
    start = np.float32(start)
    end = np.float32(end)
    step = np.float32((end - start) / np.float32(steps - 1))
    out = np.empty(steps, dtype=np.float32)
    half = steps // 2
    for i in range(steps):
        if i < half:
            out[i] = start + step * np.float32(i)
        else:
            out[i] = end - step * np.float32(steps - i - 1)
    return out


def mel_fbank(n_freqs=N_FREQ, f_min=20.0, f_max=SR // 2, n_mels=N_MELS, sample_rate=SR):
    """torchaudio.functional.melscale_fbanks(..., norm=None, mel_scale='htk'), returned transposed
    as [n_mels, n_freqs] exactly as 01-Export:102 uses it."""
    all_freqs = _linspace_f32(0, sample_rate // 2, n_freqs)
    m_min = 2595.0 * math.log10(1.0 + (f_min / 700.0))
    m_max = 2595.0 * math.log10(1.0 + (f_max / 700.0))
    m_pts = _linspace_f32(m_min, m_max, n_mels + 2)
    f_pts = (np.float32(700.0) * (np.float32(10.0) ** (m_pts / np.float32(2595.0)) - np.float32(1.0))).astype(np.float32)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts[None, :] - all_freqs[:, None]
    down = (np.float32(-1.0) * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    fb = np.maximum(np.float32(0.0), np.minimum(down, up)).astype(np.float32)
    return np.ascontiguousarray(fb.T)  # [80, 201]


def stft_basis():
    """STFT_Process.__init__ (model_definition.py:245-253): periodic Hamming window, float32
    phase `2*pi*f*t/n_fft` (the f32 phase rounding at large f*t is part of the reference numerics)."""
    # torch.hamming_window(400, periodic=True): arange(401) * (2*pi/400) -> cos -> *(-0.46) + 0.54
    n = np.arange(N_FFT, dtype=np.float32)
    window = (np.cos(n * np.float32(2.0 * math.pi / N_FFT)) * np.float32(-0.46) + np.float32(0.54)).astype(np.float32)
    f = np.arange(N_FREQ, dtype=np.int64)[:, None]
    t = np.arange(N_FFT, dtype=np.int64)[None, :]
    omega = (np.float32(2.0 * math.pi) * f.astype(np.float32)) * t.astype(np.float32) / np.float32(N_FFT)
    omega = omega.astype(np.float32)
    cos_k = (np.cos(omega) * window[None, :]).astype(np.float32)
    sin_k = (-np.sin(omega) * window[None, :]).astype(np.float32)
    return cos_k, sin_k  # [201, 400] each


def frame_counts(valid_samples, phys_samples=None):
    """Frame arithmetic: model_definition.py:286, 291-292, 317-318 and nano_onnx.py:124-127."""
    if phys_samples is None:
        phys_samples = valid_samples
    t_phys = phys_samples // HOP + 1
    t_mel_valid = valid_samples // HOP + 1
    t_lfr_valid = (t_mel_valid + LFR_N - 1) // LFR_N
    t_lfr_phys = (t_phys + LFR_N - 1) // LFR_N
    olens_1 = 1 + (t_lfr_valid - 3 + 2) // 2
    target_len = (1 + (olens_1 - 3 + 2) // 2 - 1) // 2 + 1
    return dict(t_phys=t_phys, t_mel_valid=t_mel_valid, t_lfr_valid=t_lfr_valid,
                t_lfr_phys=t_lfr_phys, target_len=target_len)


def preprocess(audio, valid):
    """F1: mean removal over valid samples, pre-emphasis, masking (model_definition.py:271-282)."""
    a = np.asarray(audio, dtype=np.float32)
    m = (np.arange(a.shape[0]) < valid).astype(np.float32)
    mean = np.float32(np.sum((a * m).astype(np.float64)) / valid)  # f32 result; sum order-free
    a = ((a - mean) * m).astype(np.float32)
    b = a.copy()
    b[1:] = a[1:] - np.float32(PRE_EMPH) * a[:-1]
    return (b * m).astype(np.float32)


def log_mel(a, cos_k=None, sin_k=None, fbank=None):
    """F2+F3: framed DFT (conv1d stride 160 on the 200/200 zero-padded signal) -> power -> mel -> log."""
    if cos_k is None:
        cos_k, sin_k = stft_basis()
    if fbank is None:
        fbank = mel_fbank()
    xp = np.pad(a, (N_FFT // 2, N_FFT // 2))
    t_phys = a.shape[0] // HOP + 1
    idx = np.arange(t_phys)[:, None] * HOP + np.arange(N_FFT)[None, :]
    frames = xp[idx].astype(np.float32)                    # [T, 400]
    re = frames @ cos_k.T                                  # [T, 201]
    im = frames @ sin_k.T
    power = (re * re + im * im).astype(np.float32)
    mel = power @ fbank.T                                  # [T, 80]
    return np.log(mel + np.float32(1e-7)).astype(np.float32)


def lfr(mel, t_mel_valid):
    """F4 LFR with replicate padding (model_definition.py:290-311). Returns x [T_lfr_phys, 560], m."""
    t_phys = mel.shape[0]
    t_lfr_valid = (t_mel_valid + LFR_N - 1) // LFR_N
    t_lfr_phys = (t_phys + LFR_N - 1) // LFR_N
    cons = mel[np.minimum(np.arange(t_phys), t_mel_valid - 1)]
    m_half = (LFR_M - 1) // 2
    right = t_lfr_phys * LFR_N + LFR_M - t_phys
    padded = np.concatenate([np.repeat(cons[:1], m_half, 0), cons, np.repeat(cons[t_phys - 1:t_phys], right, 0)], 0)
    x = np.concatenate([padded[i: i + t_lfr_phys * LFR_N: LFR_N][:t_lfr_phys] for i in range(LFR_M)], -1)
    m = (np.arange(t_lfr_phys) < t_lfr_valid).astype(np.float32)
    return (x * m[:, None]).astype(np.float32), m


def sinusoidal_pe(T, depth):
    """SinusoidalPositionEncoder.encode with positions 1..T (model_definition.py:13-28)."""
    pos = np.arange(1, T + 1, dtype=np.float32)
    inc = np.float32(np.log(np.float32(10000.0)) / np.float32(depth / 2 - 1))
    inv = np.exp(np.arange(depth // 2, dtype=np.float32) * -inc).astype(np.float32)
    st = (pos[:, None] * inv[None, :]).astype(np.float32)
    return np.concatenate([np.sin(st), np.cos(st)], -1).astype(np.float32)


def frontend(audio, valid=None):
    """Full F1-F4 for one clip: returns (x_lfr [T,560] masked, mask [T], counts)."""
    a = np.asarray(audio, dtype=np.float32)
    if valid is None:
        valid = a.shape[0]
    c = frame_counts(valid, a.shape[0])
    pre = preprocess(a, valid)
    mel = log_mel(pre)
    x, m = lfr(mel, c["t_mel_valid"])
    return x, m, c
