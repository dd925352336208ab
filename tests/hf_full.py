"""The full-dims decoder anchor (tests/golden/qwen3_full_hf.npz, make_golden.py::qwen3_full_golden): HF
Qwen3ForCausalLM at LLM_FULL on the q8_0-dequantised synthetic weights, fed the configs[1] prompt (73 prefix +
126 adaptor rows of encoder_full_60s + 5 suffix = 204 rows) and 12 greedy steps (positions 204-215).

Every decoder under test (cref, the numpy oracle, the GPU engine) quantises activations to q8_0 (ggml numerics)
where HF keeps f32, so agreement is bounded by the q8_0 noise floor (test_qwen3_q8_noise_floor): measured for cref,
cosine 0.9998 on the 8192-column sample, |logit diff| <= 0.07 on the HF top-256, argmax equal wherever the HF top-2
margin exceeds 0.07. Bars: cosine >= 0.9995, norm within 0.1 %, top-256 overlap >= 230, |diff| on the HF top-256
<= 0.15, argmax equal where the HF margin > 0.15 (two noise floors)."""
import os

import numpy as np

from conftest import GOLDEN

COS_MIN, NORM_TOL, TOP_OVERLAP_MIN, TOP_DIFF_MAX, MARGIN_ARGMAX = 0.9995, 1e-3, 230, 0.15, 0.15


def load():
    g = np.load(os.path.join(GOLDEN, "qwen3_full_hf.npz"))
    g60 = np.load(os.path.join(GOLDEN, "encoder_full_60s.npz"))
    return g, g60["adaptor"].astype(np.float32)


def prompt(g, adaptor, embed_prompt):
    """The 204-row prompt with the decoder-under-test's own fp16 embedding rows for the prefix / suffix ids."""
    return np.concatenate([embed_prompt(g["prefix_ids"]), adaptor, embed_prompt(g["suffix_ids"])], 0).astype(np.float32)


def check(g, i, lg):
    """Logits `lg` [n_vocab] of vector i (0 = prefill last row, i >= 1 = after greedy step i) against the anchor."""
    lg = np.asarray(lg, np.float64)
    a, b = lg[g["cols"]], g["col_vals"][i].astype(np.float64)
    cos = float(a @ b / np.linalg.norm(a) / np.linalg.norm(b))
    ratio = float(np.linalg.norm(lg) / g["norm"][i])
    overlap = len(set(np.argpartition(-lg, 256)[:256].tolist()) & set(g["top_ids"][i].tolist()))
    diff = float(np.abs(lg[g["top_ids"][i]] - g["top_vals"][i]).max())
    msg = f"vector {i}: cos {cos:.6f} norm ratio {ratio:.5f} top-256 overlap {overlap} max|diff| {diff:.4f}"
    assert cos >= COS_MIN and abs(ratio - 1) <= NORM_TOL and overlap >= TOP_OVERLAP_MIN and diff <= TOP_DIFF_MAX, msg
    if g["margin"][i] > MARGIN_ARGMAX:
        assert int(np.argmax(lg)) == int(g["argmax"][i]), msg + f" argmax {int(np.argmax(lg))} vs {int(g['argmax'][i])}"
    return cos
