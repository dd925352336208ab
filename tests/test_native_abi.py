"""CPU-side checks of the drop-in boundary: the in-tree libfunasr_hip.so loads and exports every
symbol include/funasr_hip.h declares (no compute calls without a GPU)."""
import os
import re

from conftest import ROOT


def test_library_exports_every_declared_symbol():
    from fun_asr_gguf import _native
    hdr = open(os.path.join(ROOT, "include", "funasr_hip.h")).read()
    declared = sorted(set(re.findall(r"\b(fa_[a-z0-9_]+)\s*\(", hdr)))
    assert declared, "no declarations parsed"
    lib = _native.load()
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(_native.EXPORTS) == declared


def test_create_without_gpu_fails_loudly():
    import pytest
    from fun_asr_gguf import _native
    from oracle import synth
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except Exception:
        pass
    with pytest.raises(RuntimeError):
        _native.Engine(synth.ENC_TINY, synth.LLM_TINY)
