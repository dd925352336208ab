"""int8-dynamic CTC graph on the GPU (Fun-ASR-Nano-CTC.int8.onnx, the reference README's default CTC model:
02-Quantize-ONNX.py:38-46) against oracle/ctc_int8.py at full CTC dims (5 blocks, vocab 60515), synthetic weights
quantised with onnxruntime's per-channel QUInt8 algorithm and uploaded as stored (fa_set_tensor_u8dq).

The integer parts (DynamicQuantizeLinear, MatMulInteger) are exact on both sides, but the graph amplifies input noise:
a per-tensor activation scale moves with the tensor's extreme value, so a 1e-7 relative perturbation of the encoder
rows moves the int8 logits by up to 0.17 and flips ids at margins up to 0.03 (1e-6: 0.20 / 0.054;
tests/test_ctc_int8.py::test_int8_ctc_noise_floor). The GPU's LayerNorm (f32 vs the oracle's float64) and bf16x3
attention are such perturbations. Bar: CTC ids equal wherever the oracle's int8 top-2 margin exceeds 0.25 (above the
measured logit movement), and at least 90 % of all ids equal. Parity against onnxruntime itself stays unpinned (absent
here)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import ctc_int8 as oi8, synth

pytestmark = pytest.mark.gpu

SR = 16000
MARGIN = 0.25


@pytest.fixture(scope="module")
def i8():
    from fun_asr_gguf import _native
    cfg = synth.ENC_FULL
    e = _native.Engine(cfg, dict(synth.LLM_TINY, n_ctx=256, max_seqs=1), max_batch=4, max_samples=SR * 62)
    e.synthetic_weights(0)
    W = synth.make_weights([t for t in synth.encoder_tensors(cfg) if t[0].startswith(("ctc_decoder.", "ctc_proj."))])
    Q = oi8.quantize_ctc(W, cfg)
    ref_f32 = e.ctc_head(np.load(os.path.join(GOLDEN, "encoder_full_10s.npz"))["enc"])
    assert not e.ctc_int8_active()
    for p, (q, sc, zp) in Q.items():
        e.set_tensor_u8dq(p + ".weight", q, sc, zp)
    assert e.ctc_int8_active()
    yield e, W, Q, ref_f32
    e.close()


def _check_ids(gpu, ref_ids, ref_lg, tag):
    top2 = np.sort(ref_lg, -1)[:, -2:]
    margin = top2[:, 1] - top2[:, 0]
    assert gpu.shape == ref_ids.shape, tag
    bad = (gpu != ref_ids) & (margin > MARGIN)
    diff = gpu != ref_ids
    print(f"{tag}: {int(diff.sum())} of {gpu.size} ids differ, max oracle margin there "
          f"{float(margin[diff].max()) if diff.any() else 0.0:.4f}")
    assert bad.sum() == 0, f"{tag}: {int(bad.sum())} non-tie CTC ids differ"
    assert diff.mean() < 0.1, f"{tag}: {int(diff.sum())} ids differ"


def test_ctc_head_int8_10s_golden_rows(i8):
    """configs[0]'s encoder rows (reference golden) through fa_ctc_head on the int8 graph."""
    e, W, Q, ref_f32 = i8
    g = np.load(os.path.join(GOLDEN, "encoder_full_10s.npz"))
    ids = e.ctc_head(g["enc"])
    ref_ids, ref_lg = oi8.ctc_ids_int8(g["enc"], W, Q, synth.ENC_FULL)
    _check_ids(ids, ref_ids, ref_lg, "10 s golden rows")
    assert (ids != ref_f32).any() or (ref_ids == g["ctc_ids"]).all()  # the int8 graph is the one that ran
    # switched off: the f32 graph again, bit for bit
    e.set_ctc_int8(False)
    try:
        assert not e.ctc_int8_active()
        assert np.array_equal(e.ctc_head(g["enc"]), ref_f32)
    finally:
        e.set_ctc_int8(True)


def test_encode_60s_int8_ctc_vs_oracle(i8):
    """configs[1] clip: the whole encode with the int8 CTC head (1001 rows, per-tensor activation scales over the
    clip's rows) against the oracle's int8 graph on the same encoder output."""
    from fun_asr_gguf.synthetic import synth_audio
    e, W, Q, _ = i8
    g = np.load(os.path.join(GOLDEN, "encoder_full_60s.npz"))
    audio = synth_audio(960000, int(g["audio_seed"]))
    out = e.encode([audio], want_enc=True)
    enc = out["enc"][0]
    assert enc.shape == (1001, 512)
    ref_ids, ref_lg = oi8.ctc_ids_int8(enc, W, Q, synth.ENC_FULL)
    _check_ids(out["ctc_ids"][0], ref_ids, ref_lg, "60 s encode")


def test_int8_ctc_batch_and_lanes_per_clip(i8):
    """Activation scales are per clip (its own [1, T, K] tensor): a ragged padded batch (incl. a < 1 s clip, whose CTC
    input is its 1 s padded length) gives each clip its own oracle result, and independent-clip lanes give exactly the
    single-clip encode's ids."""
    from fun_asr_gguf.synthetic import synth_audio
    e, W, Q, _ = i8
    clips = [synth_audio(SR * 10, 71), synth_audio(int(SR * 4.2), 72), synth_audio(int(SR * 0.8), 73)]
    out = e.encode(clips, want_enc=True)
    lanes = e.encode(clips, independent=True)
    for b, c in enumerate(clips):
        one = e.encode([c], want_enc=True)
        assert np.array_equal(lanes["ctc_ids"][b], one["ctc_ids"][0]), f"clip {b}: lanes vs single"
        ref_ids, ref_lg = oi8.ctc_ids_int8(one["enc"][0], W, Q, synth.ENC_FULL)
        _check_ids(one["ctc_ids"][0], ref_ids, ref_lg, f"clip {b} single")
        ref_ids, ref_lg = oi8.ctc_ids_int8(out["enc"][b], W, Q, synth.ENC_FULL)
        _check_ids(out["ctc_ids"][b], ref_ids, ref_lg, f"clip {b} in the padded batch")


def test_int8_ctc_invalidated_by_f32_writes(i8):
    """An f32 write to a CTC weight (fa_set_tensor_f32) or an unset of it (fa_weights_mark_unset) makes that weight's
    int8 form stale: the CTC head leaves the int8 graph (f32 again, bit for bit) until the weight is handed over as
    int8 again (the head must not keep running the old int8 weights)."""
    e, W, Q, ref_f32 = i8
    g = np.load(os.path.join(GOLDEN, "encoder_full_10s.npz"))
    int8_ids = e.ctc_head(g["enc"])
    name = next(iter(Q))
    try:
        e.set_tensor(name + ".weight", W[name + ".weight"])
        assert not e.ctc_int8_active()
        assert np.array_equal(e.ctc_head(g["enc"]), ref_f32)
        e.set_tensor_u8dq(name + ".weight", *Q[name])
        assert e.ctc_int8_active()
        e.mark_unset(name + ".weight")
        assert not e.ctc_int8_active()
    finally:
        e.set_tensor(name + ".weight", W[name + ".weight"])
        e.set_tensor_u8dq(name + ".weight", *Q[name])
    assert e.ctc_int8_active()
    assert np.array_equal(e.ctc_head(g["enc"]), int8_ids)
