"""CPU oracle for the Fun-ASR hot path — TEST INFRASTRUCTURE ONLY.

This package restates the algorithm the reference (lpyjmj/Fun-ASR-GGUF, mounted read-only at /root/reference) runs
on its per-segment hot path (`StreamDecoder.decode_stream`, fun_asr_gguf/core/decoder.py:132-246):

  frontend.py      F1-F4    model_definition.py:244-311 (+ torchaudio HTK fbank, 01-Export:102)
  encoder.py       A4-A8    model_definition.py:9-229, 313-337
  encoder_fp16.py  C5       the float16 graphs of 02-Quantize-ONNX.py:13-27
  ctc.py           A9, A14, A15  nano_ctc.py:38-232 (decode_ctc, align_timestamps), text_merge.py:14-114,
                            orchestrator.py:123-136 (segment windows)
  q8.py            q8_0 quantisation, gguf/quants.py:378-401 (bit-exact ggml reference); llama.py:778-784
  qwen3.py         A11-A13  Qwen3 decoder with ggml q8_0 x q8_0 integer-dot numerics
  bpe.py           A10      llama.cpp's qwen2 byte-level BPE tokenizer
  cref/ (cref.py)  C++/OpenMP restatement of the encoder and the decoder at full dims (also the CPU baseline)
  synth.py         deterministic synthetic weights (the repo's own spec)

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import anything from here, and only
as the checker / CPU baseline -- never as the product path.

Parity pinning: encoder/adaptor/CTC restatements against golden vectors produced by importing the reference's own
`model_definition.py` (tests/golden/make_golden.py); ctc/align/merge against the reference's own `nano_ctc.py` /
`text_merge.py`; q8 against the vendored `gguf.quants.Q8_0`. The decoder (llama.cpp b7798, absent as source) is
"parity unpinned" w.r.t. llama.cpp itself; qwen3.py and cref are anchored on HF transformers' Qwen3ForCausalLM with the
same q8_0-dequantised weights at tiny dims (tests/golden/qwen3_tiny_hf.npz, tests/test_oracle_golden.py) and at full
dims on the configs[1] prompt (tests/golden/qwen3_full_hf.npz; bars in tests/hf_full.py, tests in
tests/test_cref.py and tests/test_oracle_golden.py).
"""
