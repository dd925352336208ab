"""Generate the committed golden fixtures by running the REFERENCE's own Python in this container.

Run (container only, needs /root/reference):  python tests/golden/make_golden.py

What is imported from /root/reference/fun_asr_gguf (by file path; the package __init__ is not run
because it imports onnxruntime, which is absent):
  model_definition.py  -> encoder/adaptor/CTC golden outputs (HybridSenseVoice, EncoderExportWrapperPaddable,
                          CTCHeadExportWrapper), synthetic weights loaded via load_state_dict
  nano_ctc.py          -> decode_ctc / align_timestamps / load_ctc_tokens goldens
  text_merge.py        -> merge_transcription_results goldens
  gguf/quants.py       -> Q8_0 quantisation goldens (vendored gguf-py, declared bit-exact to ggml)
  llama.py             -> get_token_embeddings_gguf on a tiny GGUF written with the vendored GGUFWriter
Third party (not the reference): transformers Qwen3ForCausalLM as the decoder anchor (llama.cpp is absent).
The mel filterbank comes from oracle/frontend.py (torchaudio is absent) and is fed to the reference wrapper.
"""
import base64
import importlib.util
import json
import os
import sys
import tempfile
import types

import numpy as np
import torch

REF = "/root/reference/fun_asr_gguf"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fun-asr-gguf_amd"))

from oracle import synth, frontend as fe, q8  # noqa: E402
from fun_asr_gguf.synthetic import synth_audio  # noqa: E402


def load_by_path(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def ref_package_module(sub):
    """Import fun_asr_gguf.<sub> from the reference without executing its package __init__."""
    if "fun_asr_gguf_ref" not in sys.modules:
        pkg = types.ModuleType("fun_asr_gguf_ref")
        pkg.__path__ = [REF]
        import logging
        pkg.logger = logging.getLogger("fun_asr_gguf_ref")
        sys.modules["fun_asr_gguf_ref"] = pkg
        if REF not in sys.path:
            sys.path.append(REF)  # vendored gguf-py
    return importlib.import_module("fun_asr_gguf_ref." + sub)


def build_hybrid(md, cfg, seed=0):
    torch.manual_seed(0)
    h = md.HybridSenseVoice(vocab_size=cfg["ctc_vocab"])
    enc = h.audio_encoder
    enc.encoders = torch.nn.ModuleList(list(enc.encoders)[: cfg["n_blocks"] - 1])
    enc.tp_encoders = torch.nn.ModuleList(list(enc.tp_encoders)[: cfg["n_tp_blocks"]])
    h.audio_adaptor.blocks = torch.nn.ModuleList(list(h.audio_adaptor.blocks)[: cfg["adaptor_blocks"]])
    h.ctc_decoder.blocks = torch.nn.ModuleList(list(h.ctc_decoder.blocks)[: cfg["ctc_blocks"]])
    W = synth.make_weights(synth.encoder_tensors(cfg), seed)
    sd = {k: torch.from_numpy(v) for k, v in W.items()}
    missing, unexpected = h.load_state_dict(sd, strict=True), None
    h.eval()
    return h


def encoder_golden(md, cfg, audio, valid, tag, store_enc_rows=None):
    h = build_hybrid(md, cfg)
    stft = md.STFT_Process(400, 400, 160).eval()
    fbank = torch.from_numpy(fe.mel_fbank()).unsqueeze(0)
    wrap = md.EncoderExportWrapperPaddable(h, stft, fbank).eval()
    taps = {}
    hk = h.audio_encoder.register_forward_hook(lambda m, i, o: taps.__setitem__("lfr", i[0].detach().clone()))
    with torch.no_grad():
        enc, ad = wrap(torch.from_numpy(audio).view(1, 1, -1), torch.tensor([valid], dtype=torch.long))
        ctc_wrap = md.CTCHeadExportWrapper(h).eval()
        c = fe.frame_counts(valid, audio.shape[0])
        enc_valid = enc[:, : c["t_lfr_valid"]]  # CPU-EP reference feeds the unpadded enc to the CTC graph
        ids = ctc_wrap(enc_valid)
        logits = h.ctc_proj.ctc_lo(h.ctc_decoder(enc_valid, None)[0])[0]
        top2 = torch.topk(logits, 2, dim=-1).values
        margin = (top2[:, 0] - top2[:, 1]).numpy()
    hk.remove()
    tl = c["target_len"]
    rows = store_enc_rows or enc.shape[1]
    out = dict(audio=audio, valid=np.int64(valid), lfr=taps["lfr"][0].numpy(),
               enc=enc[0, :rows].numpy(), adaptor=ad[0, :tl].numpy(),
               ctc_ids=ids[0].numpy().astype(np.int32), ctc_margin=margin.astype(np.float32),
               target_len=np.int64(tl), t_lfr_valid=np.int64(c["t_lfr_valid"]))
    np.savez_compressed(os.path.join(HERE, f"encoder_{tag}.npz"), **out)
    print(f"encoder_{tag}: T={enc.shape[1]} target_len={tl} enc|max|={float(enc.abs().max()):.3f}")


def ctc_align_merge_golden(nc, tm):
    rng = np.random.default_rng(7)
    # synthetic CTC vocab with base64 tokens (01-Export: base64 token + id per line; blank = max id)
    pieces = ["你", "好", "世", "界", "的", "是", "a", "B", "c", "hello", "World", "，", "。", " ", "ok", "Xy"]
    id2tok = {i: p for i, p in enumerate(pieces)}
    blank = len(pieces)
    id2tok[blank] = "<blk>"
    with tempfile.TemporaryDirectory() as td:
        tp = os.path.join(td, "tokens.txt")
        with open(tp, "w", encoding="utf-8") as f:
            for i in range(blank + 1):
                f.write(f"{base64.b64encode(id2tok[i].encode()).decode()} {i}\n")
        loaded = nc.load_ctc_tokens(tp)
        tokens_txt = open(tp, encoding="utf-8").read()
    cases = []
    for n in [0, 1, 2, 5, 37, 167, 1001]:
        ids = rng.integers(0, blank + 1, size=n)
        ids = np.where(rng.random(n) < 0.4, blank, ids)  # plenty of blanks
        ids = np.repeat(ids, rng.integers(1, 4, size=n))[:n] if n else ids
        text, res, _ = nc.decode_ctc(ids.astype(np.int32).reshape(1, -1) if n else ids.astype(np.int32), loaded)
        cases.append(dict(ids=[int(i) for i in ids], text=text, tokens=[[r.text, r.start] for r in res]))
    # alignment cases: CTC tokens vs LLM text (mixed case, substitutions, insertions, deletions, empty)
    align_cases = []
    for k in range(12):
        n_tok = int(rng.integers(0, 40))
        toks = [(pieces[int(rng.integers(0, len(pieces)))], round(float(rng.random() * 10), 3)) for _ in range(n_tok)]
        toks.sort(key=lambda t: t[1])
        ctc_text = "".join(t for t, _ in toks)
        llm = list(ctc_text)
        for _ in range(int(rng.integers(0, 8))):
            op = int(rng.integers(0, 3))
            pos = int(rng.integers(0, len(llm) + 1))
            if op == 0:
                llm.insert(pos, pieces[int(rng.integers(0, 6))])
            elif op == 1 and llm:
                llm.pop(min(pos, len(llm) - 1))
            elif llm:
                llm[min(pos, len(llm) - 1)] = "Z"
        llm_text = "".join(llm).swapcase() if k % 3 == 0 else "".join(llm)
        if k == 5:
            llm_text = ""
        Tok = nc.Token
        al = nc.align_timestamps([Tok(t, s) for t, s in toks], llm_text)
        align_cases.append(dict(ctc=[[t, s] for t, s in toks], llm=llm_text, aligned=al))
    # merge cases: overlapping segment outputs
    merge_cases = []
    base = "今天天气很好，我们去公园散步吧。然后一起吃饭，好不好？hello world, this is a test."
    for k in range(6):
        seg_len, overlap = 20.0, [2.0, 4.0][k % 2]
        n_seg = int(rng.integers(1, 5))
        results, offsets = [], []
        for s in range(n_seg):
            off = s * (seg_len - overlap)
            a0 = int(rng.integers(0, 5)) + s * 12
            txt = base[a0 % len(base): a0 % len(base) + 18 + int(rng.integers(0, 6))]
            if k == 4 and s == 1:
                txt = ""
            segs = [{"char": ch, "start": round(j * 1.1 + float(rng.random()) * 0.1, 4)} for j, ch in enumerate(txt)]
            results.append({"text": txt, "segments": segs, "duration": seg_len})
            offsets.append(off)
        import copy
        r_in = copy.deepcopy(results)
        text, segs = tm.merge_transcription_results(copy.deepcopy(results), offsets, overlap)
        merge_cases.append(dict(results=r_in, offsets=offsets, overlap=overlap, text=text,
                                segments=[{"char": s["char"], "start": s["start"]} for s in segs]))
    with open(os.path.join(HERE, "ctc_align_merge.json"), "w", encoding="utf-8") as f:
        json.dump(dict(tokens_txt=tokens_txt, id2token={str(k): v for k, v in loaded.items()},
                       decode=cases, align=align_cases, merge=merge_cases), f, ensure_ascii=False)
    print("ctc_align_merge.json written")


def q8_golden(llama_mod):
    qs = ref_package_module("gguf.quants") if False else None
    sys.path.append(REF)
    import gguf  # vendored copy
    rng = np.random.default_rng(11)
    x = (rng.standard_normal((64, 256)) * rng.random((64, 1)) * 3).astype(np.float32)
    x[3] = 0.0  # all-zero block row -> d == 0 path
    x[5, :32] = np.linspace(-1, 1, 32, dtype=np.float32) * 127 / 2.0  # exact .5 ties -> roundf away from 0
    qb = gguf.quants.quantize(x, gguf.GGMLQuantizationType.Q8_0)
    deq = gguf.quants.dequantize(qb, gguf.GGMLQuantizationType.Q8_0)
    # tiny GGUF with a q8_0 token_embd -> reference get_token_embeddings_gguf (fp16 product rounding)
    emb = (rng.standard_normal((48, 64)) * 0.05).astype(np.float32)
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "tiny.gguf")
        w = gguf.GGUFWriter(p, "qwen3")
        w.add_embedding_length(64)
        qe = gguf.quants.quantize(emb, gguf.GGMLQuantizationType.Q8_0)
        w.add_tensor("token_embd.weight", qe, raw_dtype=gguf.GGMLQuantizationType.Q8_0)
        w.write_header_to_file(); w.write_kv_data_to_file(); w.write_tensors_to_file(); w.close()
        table = llama_mod.get_token_embeddings_gguf(p)
        gguf_bytes = open(p, "rb").read()
    np.savez_compressed(os.path.join(HERE, "q8_0.npz"), x=x, q8_bytes=qb, deq=deq, emb=emb,
                        emb_table=table, tiny_gguf=np.frombuffer(gguf_bytes, np.uint8))
    print("q8_0.npz written")


def qwen3_golden():
    """Anchor for the decoder restatement: HF Qwen3 (third party; same architecture llama.cpp runs) on
    q8_0-dequantised synthetic weights, tiny depth/vocab."""
    from transformers import Qwen3Config, Qwen3ForCausalLM
    cfg = synth.LLM_TINY
    W = synth.make_weights(synth.llm_tensors(cfg), 0)
    Wd = {}
    for k, v in W.items():
        if v.ndim == 2:
            d, q = q8.quantize_q8_0(v)
            Wd[k] = q8.dequant_f32(d, q)
        else:
            Wd[k] = v
    hc = Qwen3Config(vocab_size=cfg["n_vocab"], hidden_size=cfg["n_embd"], intermediate_size=cfg["n_ff"],
                     num_hidden_layers=cfg["n_layer"], num_attention_heads=cfg["n_head"],
                     num_key_value_heads=cfg["n_head_kv"], head_dim=cfg["head_dim"], rms_norm_eps=cfg["rms_eps"],
                     rope_theta=cfg["rope_theta"], tie_word_embeddings=True, max_position_embeddings=4096,
                     attention_bias=False, torch_dtype="float32")
    try:
        hc.rope_parameters = {"rope_type": "default", "rope_theta": cfg["rope_theta"]}
    except Exception:
        pass
    m = Qwen3ForCausalLM(hc).eval()
    sd = {"model.embed_tokens.weight": Wd["token_embd.weight"], "model.norm.weight": Wd["output_norm.weight"],
          "lm_head.weight": Wd["token_embd.weight"]}
    mp = {"attn_norm": "input_layernorm", "ffn_norm": "post_attention_layernorm", "attn_q": "self_attn.q_proj",
          "attn_k": "self_attn.k_proj", "attn_v": "self_attn.v_proj", "attn_output": "self_attn.o_proj",
          "attn_q_norm": "self_attn.q_norm", "attn_k_norm": "self_attn.k_norm", "ffn_gate": "mlp.gate_proj",
          "ffn_up": "mlp.up_proj", "ffn_down": "mlp.down_proj"}
    for l in range(cfg["n_layer"]):
        for g, h in mp.items():
            sd[f"model.layers.{l}.{h}.weight"] = Wd[f"blk.{l}.{g}.weight"]
    m.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}, strict=True)
    rng = np.random.default_rng(5)
    ids = rng.integers(0, cfg["n_vocab"], size=20)
    d, q = q8.quantize_q8_0(W["token_embd.weight"])
    prompt = np.concatenate([q8.dequant_numpy_f16(d[ids[:12]], q[ids[:12]]),
                             (rng.standard_normal((8, cfg["n_embd"])) * 0.05).astype(np.float32)], 0)
    with torch.no_grad():
        out = m(inputs_embeds=torch.from_numpy(prompt)[None]).logits[0].numpy()
        seq = []
        emb = torch.from_numpy(prompt)[None]
        for _ in range(6):
            lg = m(inputs_embeds=emb).logits[0, -1]
            t = int(torch.argmax(lg))
            seq.append(t)
            e = torch.from_numpy(q8.dequant_f32(d[[t]], q[[t]]))[None]
            emb = torch.cat([emb, e], 1)
    np.savez_compressed(os.path.join(HERE, "qwen3_tiny_hf.npz"), prompt=prompt, logits=out, greedy=np.array(seq))
    print("qwen3_tiny_hf.npz written; greedy", seq)


def main():
    torch.set_num_threads(8)
    md = load_by_path("ref_model_definition", os.path.join(REF, "model_definition.py"))
    nc = load_by_path("ref_nano_ctc", os.path.join(REF, "nano_ctc.py"))
    tm = load_by_path("ref_text_merge", os.path.join(REF, "text_merge.py"))
    llama_mod = ref_package_module("llama")
    ctc_align_merge_golden(nc, tm)
    q8_golden(llama_mod)
    a10 = synth_audio(160000, 0)
    a3 = synth_audio(52817, 3)
    encoder_golden(md, synth.ENC_TINY, a3, 52817, "tiny_3s")
    # padded batch semantics (DML path): 2.0 s valid inside a 3.3 s physical buffer
    pad = np.zeros(52817, np.float32)
    pad[:32000] = a3[:32000]
    encoder_golden(md, synth.ENC_TINY, pad, 32000, "tiny_pad2s")
    encoder_golden(md, synth.ENC_FULL, a10, 160000, "full_10s")
    qwen3_golden()


if __name__ == "__main__":
    main()
