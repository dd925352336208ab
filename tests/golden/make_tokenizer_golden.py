"""Generate the tokenizer fixtures (container only): python tests/golden/make_tokenizer_golden.py

No real Qwen3 GGUF ships with the reference (weights absent), so a synthetic Qwen2-style byte-level BPE
is trained here with HuggingFace `tokenizers` (third party: the library Qwen's tokenizer.json runs on), configured
as Qwen2/Qwen3's tokenizer.json is (Split on the Qwen2 regex, isolated; ByteLevel without prefix space or regex;
<|endoftext|> <|im_start|> <|im_end|> as special added tokens). It is written to a GGUF with the reference's own
vendored gguf-py GGUFWriter (/root/reference/fun_asr_gguf/gguf), with the metadata layout convert_hf_to_gguf.py's
_set_vocab_gpt2 produces (:1283-1291): tokenizer.ggml.model gpt2, pre qwen2, tokens, token_type (special -> 3
CONTROL), merges, eos id. The expected ids / pieces come from `tokenizers` itself.
Outputs: tests/golden/tokenizer_qwen2_synth.gguf, tests/golden/tokenizer_golden.json
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
sys.path.append("/root/reference/fun_asr_gguf")  # vendored gguf-py

import gguf  # noqa: E402
from tokenizers import AddedToken, Regex, Tokenizer, decoders, models, pre_tokenizers, trainers  # noqa: E402

from fun_asr_gguf.prompt_utils import prompt_texts  # noqa: E402
from oracle.bpe import QWEN2_PRETOKENIZE, bytes_to_unicode  # noqa: E402

SPECIALS = ["<|endoftext|>", "<|im_start|>", "<|im_end|>"]


def corpus():
    zh = ("今天天气很好，我们去公园散步吧。然后一起吃饭，好不好？语音转写任务需要结合上下文信息，更加准确地完成。"
          "热词列表包括人工智能、深度学习、语音识别、大模型推理。北京上海广州深圳，二零二四年十月十六日。")
    en = ("Hello world, this is a test. I'm sure we'll see; don't worry, they've done it and you'd know. "
          "The quick brown fox jumps over the lazy dog 1234567890 times!!! Speech recognition on MI355X GPUs.")
    mixed = "混合 English 和中文 text，数字 2024 年 3.14 和 100%。\n\n新的一段\r\n\ttab 缩进   多个空格  "
    lines = [zh, en, mixed, prompt_texts()[0], prompt_texts(["阿里巴巴", "通义千问"], "中文", "会议记录")[0],
             prompt_texts()[1]]
    return [ln for ln in lines for _ in range(20)]


def build():
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(QWEN2_PRETOKENIZE), behavior="isolated", invert=False),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    tok.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=1200, min_frequency=2, initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                             special_tokens=[AddedToken(s, special=True, normalized=False) for s in SPECIALS],
                             show_progress=False)
    tok.train_from_iterator(corpus(), trainer=tr)
    return tok


def main():
    tok = build()
    model = json.loads(tok.to_str())["model"]
    vocab = model["vocab"]
    merges = [" ".join(m) if isinstance(m, list) else m for m in model["merges"]]
    tokens = [None] * len(vocab)
    for t, i in vocab.items():
        tokens[i] = t
    assert None not in tokens
    types = [3 if t in SPECIALS else 1 for t in tokens]
    path = os.path.join(HERE, "tokenizer_qwen2_synth.gguf")
    w = gguf.GGUFWriter(path, "qwen3")
    w.add_tokenizer_model("gpt2")
    w.add_tokenizer_pre("qwen2")
    w.add_token_list(tokens)
    w.add_token_types(types)
    w.add_token_merges(merges)
    w.add_eos_token_id(vocab["<|im_end|>"])
    w.write_header_to_file()
    w.write_kv_data_to_file()
    w.write_tensors_to_file()
    w.close()
    texts = [prompt_texts()[0], prompt_texts()[1], prompt_texts(["阿里巴巴", "通义千问", "MI355X"], None, None)[0],
             prompt_texts(None, "英文", "上次会议讨论了 GPU 推理。")[0],
             "I'm sure we'll see; don't worry, THEY'VE done it, you'D know. It's 'quoted'.",
             "数字 2024 年 3.14159 和 100%，１２３ 全角数字。", "a  b\n\n c\t\td  \n", "   leading and trailing   ",
             "emoji 😀🚀 and symbols ©®™ — “quotes” «guillemets»", "!!!???...,,,;;; ---", "line1\r\nline2\rline3\n",
             "<|im_start|>user\n你好<|im_end|>\n<|im_start|>assistant\n", "<|im_end|><|im_end|>", "",
             "unseen words: xylophone quizzical 魑魅魍魉", "tab\tseparated\tvalues\t\t", "\n\n\n", " ", "x",
             "Mixed中English混合text123数字"]
    cases = [{"text": t, "ids": tok.encode(t, add_special_tokens=False).ids} for t in texts]
    u2b = {v: k for k, v in bytes_to_unicode().items()}
    pieces = {}
    for i in list(range(0, len(tokens), 7)) + [vocab[s] for s in SPECIALS]:
        t = tokens[i]
        pieces[str(i)] = list(t.encode("utf-8")) if t in SPECIALS else [u2b[c] for c in t]
    json.dump({"n_vocab": len(tokens), "eos": vocab["<|im_end|>"], "specials": {s: vocab[s] for s in SPECIALS},
               "cases": cases, "pieces": pieces}, open(os.path.join(HERE, "tokenizer_golden.json"), "w"),
              ensure_ascii=False, indent=0)
    print(f"{path}: {len(tokens)} tokens, {len(merges)} merges; {len(cases)} cases")


if __name__ == "__main__":
    main()
