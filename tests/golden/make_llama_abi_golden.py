"""Golden ABI facts of the reference's llama.cpp bindings -> tests/golden/llama_abi.json.

Imports the reference's own fun_asr_gguf/llama.py (by path, without its package __init__, which needs onnxruntime) and
records what a library standing in its bin/ directory must provide:
  * the ctypes struct layouts it declares for llama.cpp b7798 (llama.py:27-104): size and per-field offset / size;
  * the exported symbols it binds (llama.<name> / ggml.<name> in init_llama_lib, llama.py:186-346), read from the
    module's source text.
tests/test_llama_compat.py checks include/llama_compat.h's structs (fa_llama_struct_sizes) and the built libraries'
exports against it. Run in this container (the reference is absent on the GPU box):
    python tests/golden/make_llama_abi_golden.py
"""
import ctypes
import importlib
import inspect
import json
import logging
import os
import re
import sys
import types

REF = "/root/reference/fun_asr_gguf"
HERE = os.path.dirname(os.path.abspath(__file__))


def ref_llama():
    if "fun_asr_gguf_ref" not in sys.modules:
        pkg = types.ModuleType("fun_asr_gguf_ref")
        pkg.__path__ = [REF]
        pkg.logger = logging.getLogger("fun_asr_gguf_ref")
        sys.modules["fun_asr_gguf_ref"] = pkg
        if REF not in sys.path:
            sys.path.append(REF)  # vendored gguf-py
    return importlib.import_module("fun_asr_gguf_ref.llama")


def layout(cls):
    return {"size": ctypes.sizeof(cls),
            "fields": [[name, getattr(cls, name).offset, getattr(cls, name).size] for name, _ in cls._fields_]}


def main():
    m = ref_llama()
    structs = {n: layout(getattr(m, n)) for n in ("llama_model_params", "llama_context_params",
                                                   "llama_sampler_chain_params", "llama_logit_bias", "llama_batch")}
    src = inspect.getsource(m.init_llama_lib)
    symbols = {"libllama.so": sorted(set(re.findall(r"\bllama\.(llama_\w+)", src))),
               "libggml.so": sorted(set(re.findall(r"\bggml\.(ggml_\w+)", src)))}
    out = {"source": "fun_asr_gguf/llama.py (llama.cpp b7798 bindings)", "structs": structs, "symbols": symbols}
    with open(os.path.join(HERE, "llama_abi.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(symbols))


if __name__ == "__main__":
    main()
