import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


def _ensure_cref():
    """oracle/_build/libcref.so (the C++ oracle) is built by __graft_entry__.build(); build it here when missing
    (CPU container only: the GPU box receives the prebuilt library with the tree)."""
    import shutil
    import subprocess
    lib = os.path.join(ROOT, "oracle", "_build", "libcref.so")
    src = os.path.join(ROOT, "oracle", "cref", "cref.cpp")
    stale = not os.path.exists(lib) or os.path.getmtime(lib) < os.path.getmtime(src)
    if stale and shutil.which("make") and shutil.which("g++"):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=False)


_ensure_cref()
