"""Model dimensions. FULL = Fun-ASR-Nano-2512 (SenseVoiceEncoderSmall + adaptor + CTC head,
/root/reference/fun_asr_gguf/model_definition.py:191-229; Qwen3-0.6B decoder, 03-Export-Decoder-GGUF.py).
TINY keeps every width and shrinks only depths/vocabularies (tests, smoke)."""

ENC_FULL = dict(n_mels=80, lfr_m=7, lfr_n=6, d_in=560, d_model=512, n_heads=4, d_ffn=2048, n_blocks=50,
                n_tp_blocks=20, fsmn_k=11, d_llm=1024, adaptor_ffn=2048, adaptor_blocks=2, adaptor_heads=8,
                ctc_blocks=5, ctc_heads=8, ctc_ffn=2048, ctc_vocab=60515)
LLM_FULL = dict(n_layer=28, n_embd=1024, n_head=16, n_head_kv=8, head_dim=128, n_ff=3072, n_vocab=151936,
                rope_theta=1000000.0, rms_eps=1e-6)
ENC_TINY = dict(ENC_FULL, n_blocks=3, n_tp_blocks=2, adaptor_blocks=1, ctc_blocks=1, ctc_vocab=3001)
LLM_TINY = dict(LLM_FULL, n_layer=2, n_vocab=4096)

MODELS = {"full": (ENC_FULL, LLM_FULL), "tiny": (ENC_TINY, LLM_TINY)}
