"""Prompt construction (PromptBuilder.build_prompt, /root/reference/fun_asr_gguf/prompt_utils.py:16-54).

Same prefix/suffix text; the tokens are turned into embedding rows on the GPU with the numpy-f16 product
rounding of the reference's cached table (llama.py:782-784) via fa_embd_rows(fp16_round=1).
"""
from typing import List, Optional, Tuple

import numpy as np

SYSTEM_PREFIX = "<|im_start|>system\nYou are a helpful assistant.<|im_end|>\n<|im_start|>user\n"
SUFFIX = "<|im_end|>\n<|im_start|>assistant\n"


def prompt_texts(hotwords: Optional[List[str]] = None, language: Optional[str] = None,
                 context: Optional[str] = None) -> Tuple[str, str]:
    p = SYSTEM_PREFIX
    if hotwords or context:
        if context:
            p += "请结合上下文信息，更加准确地完成语音转写任务。\n\n\n"
            p += f"**上下文信息：**{context}\n\n\n"
        if hotwords:
            p += f"热词列表：[{', '.join(hotwords)}]\n"
    p += "语音转写：" if not language else f"语音转写成{language}："
    return p, SUFFIX


class PromptBuilder:
    def __init__(self, vocab, engine):
        self.vocab = vocab
        self.engine = engine
        self.fixed_ids = None  # benchmark protocol: (prefix_ids, suffix_ids) pinned when no tokenizer exists
        # embedding rows of recent prompts (a batch's streams usually share one prompt): keyed by the engine object,
        # its weight generation and the token ids, so a weight change or a new engine never serves stale rows
        self._embd_cache = {}

    def build_ids(self, hotwords=None, language=None, context=None):
        p, s = prompt_texts(hotwords, language, context)
        if self.fixed_ids is not None:
            return list(self.fixed_ids[0]), list(self.fixed_ids[1]), p
        return self.vocab.tokenize(p), self.vocab.tokenize(s), p

    def build_prompt(self, hotwords=None, language=None, context=None):
        """-> (prefix_embd, suffix_embd, n_prefix, n_suffix, prefix_text), like the reference."""
        pi, si, p = self.build_ids(hotwords, language, context)
        gen = getattr(self.engine, "weights_gen", None)
        key = (id(self.engine), gen, tuple(pi), tuple(si))
        hit = self._embd_cache.get(key) if gen is not None else None
        if hit is None:
            E = int(self.engine.llm_cfg["n_embd"]) if hasattr(self.engine, "llm_cfg") else 1024
            pe = self.engine.embd_rows(np.array(pi, np.int32), fp16_round=True) if pi else np.zeros((0, E), np.float32)
            se = self.engine.embd_rows(np.array(si, np.int32), fp16_round=True) if si else np.zeros((0, E), np.float32)
            pe.flags.writeable = False  # shared by every caller of this prompt: read-only
            se.flags.writeable = False
            hit = (pe, se)
            if gen is not None:  # an engine without a weight generation cannot tell stale rows: no caching
                if len(self._embd_cache) >= 64:
                    self._embd_cache.clear()
                self._embd_cache[key] = hit
        pe, se = hit
        return pe, se, len(pi), len(si), p
