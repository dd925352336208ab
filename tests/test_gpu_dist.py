"""The result gather over RCCL (backend "nccl") on the GPU box: one rank per GPU, so a one-GPU box runs world_size 1
(RCCL refuses two ranks on one device). It exercises the real collective path of `parallel.gather_to_root`
(two tensor all_gathers of the JSON records over RCCL on the rank's device) and the real engine through `transcribe(..., ranks=dist)`; the N > 1
logic is covered on CPU by tests/test_distributed_gloo.py (world_size 2, gloo)."""
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "fun-asr-gguf_amd"), os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        from test_distributed_gloo import _StubOrch
        from fun_asr_gguf.parallel import sharded_decode
        chunks = [[0.0] * n for n in (960, 960, 320)]
        stub = sharded_decode(_StubOrch(), chunks, None, None, False, 0.0, 1.0, 50, dist)
        stub = [(r.text, r.aligned) for r in stub]
        from fun_asr_gguf import create_asr_engine
        from fun_asr_gguf.synthetic import synth_audio
        eng = create_asr_engine("synthetic", "synthetic", "synthetic", "synthetic", verbose=False, model="tiny",
                                max_batch=4, n_ctx=512, n_predict=8, ignore_eos=True)
        audio = synth_audio(16000 * 14, 77)
        a = eng.transcribe(audio, segment_size=6.0, overlap=2.0, temperature=0.0, verbose=False, ranks=dist)
        b = eng.transcribe(audio, segment_size=6.0, overlap=2.0, temperature=0.0, verbose=False)
        eng.cleanup()
        q.put((stub, a.text == b.text, a.segments == b.segments))
    finally:
        dist.destroy_process_group()


def test_rccl_gather_world1():
    from test_distributed_gloo import _StubOrch
    from fun_asr_gguf.parallel import from_record, to_record
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    stub, same_text, same_segments = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    single = [from_record(to_record(d)) for d in _StubOrch().decode_segments([[0.0] * n for n in (960, 960, 320)])]
    assert stub == [(r.text, r.aligned) for r in single]
    assert same_text and same_segments


def _native_worker(port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "fun-asr-gguf_amd"), os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=0, world_size=1)  # bootstrap only: the records move through the engine's RCCL
    try:
        from fun_asr_gguf import create_asr_engine
        from fun_asr_gguf.parallel import init_native_comm
        from fun_asr_gguf.synthetic import synth_audio
        eng = create_asr_engine("synthetic", "synthetic", "synthetic", "synthetic", verbose=False, model="tiny",
                                max_batch=4, n_ctx=512, n_predict=8, ignore_eos=True)
        e = eng.models.engine
        init_native_comm(e, dist)
        blobs = [e.comm_allgather(b"records of rank 0 \xe4\xb8\xad"), e.comm_allgather(b""), e.comm_allgather(b"x" * 70000)]
        audio = synth_audio(16000 * 14, 77)
        a = eng.transcribe(audio, segment_size=6.0, overlap=2.0, temperature=0.0, verbose=False, ranks=dist)
        b = eng.transcribe(audio, segment_size=6.0, overlap=2.0, temperature=0.0, verbose=False)
        eng.cleanup()
        q.put((blobs, a.text == b.text, a.segments == b.segments, bool(a.text)))
    finally:
        dist.destroy_process_group()


def test_engine_native_rccl_gather_world1():
    """The engine's own RCCL communicator (fa_comm_init, bootstrapped over a gloo group): byte records round-trip through
    the two all-gathers (empty and 70 KB ones included), and transcribe(ranks=) gathers through it (parallel.py
    gather_native) with the result of the unsharded call."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_native_worker, args=(_free_port(), q))
    p.start()
    blobs, same_text, same_segments, nonempty = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert blobs == [[b"records of rank 0 \xe4\xb8\xad"], [b""], [b"x" * 70000]]
    assert same_text and same_segments and nonempty
