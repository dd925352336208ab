"""Segment/clip data parallelism across the GPUs of one node.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on ROCm, "gloo" in CPU tests).
Segments are assigned longest-first to the least-loaded rank (LPT); every rank decodes its share as one
device batch; the only exchange is the result gather to rank 0 (all-gathers of the JSON-encoded per-segment
records: text, char timestamps, hotwords, CTC tokens, timings), after which rank 0 merges. The gather runs through the
engine's own RCCL communicator when one was set up (init_native_comm -> fa_comm_*), else through torch.distributed.
No data-path collective: the PCM chunks are cut from the same input on every rank.
"""
import json
from dataclasses import asdict

from .nano_ctc import Token
from .nano_dataclass import DecodeResult, Timings


def lpt_assign(lengths, world):
    """Longest-processing-time-first: -> list of index lists, one per rank (deterministic)."""
    order = sorted(range(len(lengths)), key=lambda i: (-lengths[i], i))
    load = [0.0] * world
    out = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        out[r].append(i)
        load[r] += lengths[i]
    return [sorted(x) for x in out]


def to_record(d):
    return dict(text=d.text, aligned=d.aligned, hotwords=d.hotwords, n_gen=d.n_gen, is_aborted=d.is_aborted,
                ctc=[(t.text, t.start) for t in (d.ctc_results or [])], timings=asdict(d.timings),
                n_prefix=d.n_prefix, n_suffix=d.n_suffix)


def from_record(r):
    return DecodeResult(text=r["text"], aligned=r["aligned"], hotwords=r["hotwords"], n_gen=r["n_gen"],
                        is_aborted=r["is_aborted"], ctc_results=[Token(t, s) for t, s in r["ctc"]],
                        timings=Timings(**r["timings"]), n_prefix=r["n_prefix"], n_suffix=r["n_suffix"])


def _pack(records_by_index):
    """Records -> UTF-8 JSON bytes (floats in shortest round-trip form: the merge on rank 0 sees the exact values)."""
    return json.dumps(sorted(records_by_index.items()), ensure_ascii=False).encode("utf-8")


def init_native_comm(engine, dist, group=None):
    """Give `engine` its own RCCL communicator over the ranks of `dist` (fa_comm_init): rank 0 creates the 128-byte id
    and broadcasts it over `dist` (any backend: it is only the bootstrap). Afterwards gather_to_root moves the records
    through the engine (native RCCL all-gathers over xGMI), not through torch.distributed."""
    import torch
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    uid = torch.zeros(128, dtype=torch.uint8, device=dev)
    if rank == 0:
        uid.copy_(torch.frombuffer(bytearray(engine.comm_unique_id()), dtype=torch.uint8))
    dist.broadcast(uid, 0, group=group)
    engine.comm_init(rank, world, bytes(uid.cpu().numpy()))
    return engine


def _merge(blobs, n_total):
    merged = {}
    for b in blobs:
        for idx, rec in json.loads(b.decode("utf-8")):
            merged[int(idx)] = rec
    assert len(merged) == n_total, f"gather lost segments: {len(merged)} of {n_total}"
    return [merged[i] for i in range(n_total)]


def gather_native(records_by_index, n_total, engine):
    """gather_to_root through the engine's own RCCL communicator (init_native_comm): every rank's JSON records,
    merged on rank 0."""
    blobs = engine.comm_allgather(_pack(records_by_index))
    return _merge(blobs, n_total) if engine.comm_rank == 0 else None


def gather_to_root(records_by_index, n_total, dist, group=None):
    """records_by_index: {segment index: record} of this rank -> full ordered list on rank 0, None elsewhere.
    Two tensor collectives over the process group (RCCL over xGMI with backend "nccl": device tensors; gloo: host): an
    all_gather of the payload sizes, then an all_gather of the JSON payloads padded to the largest (KB-scale: latency-
    bound). No pickling: the records cross as UTF-8 JSON."""
    import torch
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    payload = _pack(records_by_index)
    size = torch.tensor([len(payload)], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, size, group=group)
    sizes = [int(x.item()) for x in sizes]
    n = max(1, max(sizes))
    buf = torch.zeros(n, dtype=torch.uint8, device=dev)
    if payload:
        buf[:len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(dev)
    bufs = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.all_gather(bufs, buf, group=group)
    if rank != 0:
        return None
    return _merge([bytes(b[:k].cpu().numpy()) for b, k in zip(bufs, sizes)], n_total)


def sharded_decode(orch, chunks, language, context, verbose, temperature, top_p, top_k, dist):
    """Decode `chunks` across the ranks of `dist` (the torch.distributed module, initialised)."""
    world, rank = dist.get_world_size(), dist.get_rank()
    mine = lpt_assign([len(c) for c in chunks], world)[rank]
    local = orch.decode_segments([chunks[i] for i in mine], language, context, verbose, temperature, top_p,
                                 top_k) if mine else []
    recs = {i: to_record(d) for i, d in zip(mine, local)}
    eng = getattr(getattr(orch, "models", None), "engine", None)
    if getattr(eng, "comm_world", 0) == world:  # the engine's own RCCL communicator (init_native_comm)
        full = gather_native(recs, len(chunks), eng)
    else:
        full = gather_to_root(recs, len(chunks), dist)
    return None if full is None else [from_record(r) for r in full]
