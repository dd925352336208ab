"""CPU oracle for the Fun-ASR hot path — TEST INFRASTRUCTURE ONLY.

This package restates, in numpy, the algorithm the reference (lpyjmj/Fun-ASR-GGUF,
mounted read-only at /root/reference) runs on its per-segment hot path
(`StreamDecoder.decode_stream`, fun_asr_gguf/core/decoder.py:132-246):

  frontend.py  F1-F4  model_definition.py:244-311 (+ torchaudio HTK fbank, 01-Export:102)
  encoder.py   A4-A8  model_definition.py:9-229, 313-337
  ctc.py       A9     nano_ctc.py:38-116
  align.py     A14    nano_ctc.py:118-232
  merge.py     A15    text_merge.py:14-114, orchestrator.py:123-189
  q8.py        q8_0 quantisation, gguf/quants.py:378-401 (bit-exact ggml reference)
  qwen3.py     A11-A13 Qwen3 decoder with ggml q8_0 x q8_0 integer-dot numerics
  synth.py     deterministic synthetic weights (the repo's own spec)

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import
anything from here, and only as the checker / CPU baseline -- never as the product path.

Parity pinning: encoder/adaptor/CTC restatements are pinned against golden vectors
produced by importing the reference's own `model_definition.py` (tests/golden/make_golden.py);
ctc/align/merge against the reference's own `nano_ctc.py` / `text_merge.py`; q8 against the
vendored `gguf.quants.Q8_0`. The decoder (llama.cpp b7798, absent as source) is
"parity unpinned" w.r.t. llama.cpp; it is anchored on HF transformers' Qwen3 with the
same q8_0-dequantised weights (tolerance stated in tests/test_oracle_qwen3.py).
"""
