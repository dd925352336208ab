"""N>1 result-gather path on CPU: world_size 2 with the gloo backend. Each rank 'decodes'
its LPT share (stub decode, no GPU), records are gathered to rank 0 and merged; rank 0 must see exactly
the records of a single-rank run."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _StubOrch:
    def decode_segments(self, chunks, *a):
        from fun_asr_gguf.nano_ctc import Token
        from fun_asr_gguf.nano_dataclass import DecodeResult
        out = []
        for c in chunks:
            n = len(c)
            txt = "".join(chr(0x4E00 + (n + k) % 50) for k in range(5))
            out.append(DecodeResult(text=txt, aligned=[{"char": ch, "start": k * 0.1} for k, ch in enumerate(txt)],
                                    ctc_results=[Token(txt[:2], 0.0)], hotwords=[]))
        return out


class _FakeCommEngine:
    """The engine's fa_comm_* surface (comm_rank / comm_world / comm_allgather) over the gloo group: exercises
    parallel.gather_native's protocol at world > 1 on CPU (the RCCL collectives themselves run in tests/test_gpu_dist.py)."""

    def __init__(self, dist):
        self.dist, self.comm_rank, self.comm_world = dist, dist.get_rank(), dist.get_world_size()
        self.calls = 0

    def comm_allgather(self, payload):
        self.calls += 1
        out = [None] * self.comm_world
        self.dist.all_gather_object(out, bytes(payload))
        return out


def _native_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "fun-asr-gguf_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fun_asr_gguf.parallel import sharded_decode
    orch = _StubOrch()
    orch.models = type("M", (), {})()
    orch.models.engine = _FakeCommEngine(dist)
    chunks = [[0.0] * n for n in (960, 960, 960, 960, 960, 320)]
    res = sharded_decode(orch, chunks, None, None, False, 0.0, 1.0, 50, dist)
    assert orch.models.engine.calls == 1
    if rank == 0:
        q.put([(r.text, r.aligned, [(t.text, t.start) for t in r.ctc_results]) for r in res])
    else:
        assert res is None
    dist.barrier()
    dist.destroy_process_group()


def test_native_gather_protocol_world3():
    """sharded_decode through the engine's own communicator (parallel.gather_native) at world 3: rank 0 gets exactly
    the single-rank records."""
    from fun_asr_gguf.parallel import to_record, from_record
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_native_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = [from_record(to_record(d)) for d in _StubOrch().decode_segments([[0.0] * n for n in (960, 960, 960, 960, 960, 320)])]
    assert got == [(r.text, r.aligned, [(t.text, t.start) for t in r.ctc_results]) for r in single]


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "fun-asr-gguf_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fun_asr_gguf.parallel import sharded_decode
    chunks = [[0.0] * n for n in (960, 960, 960, 960, 960, 320)]
    res = sharded_decode(_StubOrch(), chunks, None, None, False, 0.0, 1.0, 50, dist)
    if rank == 0:
        q.put([(r.text, r.aligned, [(t.text, t.start) for t in r.ctc_results]) for r in res])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gather_world2_equals_single(world):
    """world 2 and 3 (uneven LPT shares: 6 segments over 3 ranks, one rank with the short one) and 8 (the driver's
    8-GPU C4 shape: 6 segments over 8 ranks, two ranks with no segment)."""
    from fun_asr_gguf.parallel import to_record, from_record
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = [from_record(to_record(d)) for d in _StubOrch().decode_segments([[0.0] * n for n in (960, 960, 960, 960, 960, 320)])]
    assert got == [(r.text, r.aligned, [(t.text, t.start) for t in r.ctc_results]) for r in single]


def _api_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "fun-asr-gguf_amd"), os.path.join(root, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fake_engine import fake_api
    from fun_asr_gguf.synthetic import synth_audio
    api = fake_api(max_batch=2)
    audio = synth_audio(16000 * 300, 4000)
    res = api.transcribe(audio, segment_size=60.0, overlap=4.0, temperature=0.0, verbose=False, ranks=dist)
    clips = [synth_audio(16000 * s, 100 + i) for i, s in enumerate((60, 12, 45, 60, 3, 33, 59))]
    batch = api.transcribe_batch(clips, temperature=0.0, ranks=dist)
    if rank == 0:
        q.put((res.text, res.segments, res.ctc_text, [(d.text, d.aligned, d.n_gen) for d in batch]))
    else:
        assert batch is None
    dist.barrier()
    dist.destroy_process_group()


def test_transcribe_and_batch_sharded_world2_through_real_orchestrator():
    """The real TranscriptionOrchestrator / StreamDecoder / merge on a host fake engine (tests/fake_engine.py):
    C4-style 300 s file (6 segments, LPT over 2 ranks + gather_object + merge on rank 0) and a 7-clip
    transcribe_batch(ranks=) both equal the single-rank run exactly."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "tests")]
    from fake_engine import fake_api
    from fun_asr_gguf.synthetic import synth_audio
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_api_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    api = fake_api(max_batch=2)
    audio = synth_audio(16000 * 300, 4000)
    res = api.transcribe(audio, segment_size=60.0, overlap=4.0, temperature=0.0, verbose=False)
    clips = [synth_audio(16000 * s, 100 + i) for i, s in enumerate((60, 12, 45, 60, 3, 33, 59))]
    batch = api.transcribe_batch(clips, temperature=0.0)
    assert res.text and len(res.segments) > 0
    assert got == (res.text, res.segments, res.ctc_text, [(d.text, d.aligned, d.n_gen) for d in batch])
