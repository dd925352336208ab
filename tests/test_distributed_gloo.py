"""N>1 result-gather path on CPU: world_size 2 with the gloo backend. Each rank 'decodes'
its LPT share (stub decode, no GPU), records are gathered to rank 0 and merged; rank 0 must see exactly
the records of a single-rank run."""
import os
import socket

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


def test_gather_world2_equals_single():
    from fun_asr_gguf.parallel import to_record, from_record
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = [from_record(to_record(d)) for d in _StubOrch().decode_segments([[0.0] * n for n in (960, 960, 960, 960, 960, 320)])]
    assert got == [(r.text, r.aligned, [(t.text, t.start) for t in r.ctc_results]) for r in single]
