"""Benchmark of the Fun-ASR hot path on MI355X (BASELINE.json metric: RTF and audio-sec/s/GPU on 60 s
16 kHz clips). Workload = configs[1]: one 60 s clip per step per GPU through the full product path
(FunASREngine.decode_stream: GPU frontend + fp32 encoder + adaptor + CTC head/argmax/collapse, prompt,
q8_0 Qwen3 prefill of 73 + 126 + 5 tokens, 253 greedy decode steps with EOS ignored, native alignment).
Synthetic seeded audio and synthetic weights of the full architecture (no checkpoints ship).

  python bench.py [--gpus N --steps K --warmup W]
  N>1, either form:
    python bench.py --gpus N ...          (this script spawns N rank processes itself, before any GPU call)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Prints ONE JSON line on rank 0. value = total audio seconds of all ranks / max-over-ranks wall time of the
K timed steps (inputs resident in HBM: fa_pcm_upload before the timed region). n_gpus = the RCCL world size.
"""
import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]

import numpy as np  # noqa: E402

CLIP_S = 60.0
SR = 16000
N_PREFIX, N_SUFFIX, N_GEN = 73, 5, 253   # README.md:244-268 (204 input tokens, 253 generated)
HBM_PEAK_GBS = 8000.0                    # MI355X_MICROARCH.md chip table (spec)
FP32_MFMA_PEAK_TFS = 157.3                # v_mfma_f32_32x32x2_f32, dense
BF16X3_PEAK_TFS = 2500.0 / 3.0           # bf16 dense 2.5 PF/s, three bf16 products per f32-equivalent product


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv, script=None, grace_s=30.0):
    """`python bench.py --gpus N` without a launcher: start N fresh rank processes of `script` (default this file)
    with torchrun's environment (RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR 127.0.0.1 /
    MASTER_PORT), one GPU each (the rank binds device LOCAL_RANK). The parent imports no torch and makes no GPU call
    (a process that has initialised HIP must not start GPU children by exec, and needs no device here). Rank 0's
    stdout (the JSON line) is returned; the other ranks' stdout and every rank's stderr pass through to stderr. When a
    rank fails, the others get `grace_s` to exit (a peer blocked in a collective never will) and are then killed by
    PID. -> (worst exit code, rank 0's stdout)."""
    script = script or os.path.abspath(__file__)
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), BENCH_LAUNCHER="spawn")
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr, stderr=None))
    out0 = []
    import threading
    reader = threading.Thread(target=lambda: out0.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    failed_at = None
    while True:
        rcs = [p.poll() for p in procs]
        if all(rc is not None for rc in rcs):
            break
        if failed_at is None and any(rc not in (None, 0) for rc in rcs):
            failed_at = time.monotonic()
            log(f"bench launcher: rank(s) {[r for r, rc in enumerate(rcs) if rc not in (None, 0)]} failed")
        if failed_at is not None and time.monotonic() - failed_at > grace_s:
            for p, rc in zip(procs, rcs):
                if rc is None:
                    p.send_signal(signal.SIGKILL)
        time.sleep(0.2)
    reader.join(timeout=10)
    rcs = [p.returncode for p in procs]
    worst = max(rcs, key=lambda rc: (rc != 0, abs(rc)))
    text = out0[0].decode("utf-8", "replace") if out0 and out0[0] else ""
    return worst, text


def cpu_baseline():
    """The C2 workload UNEXTRAPOLATED on the host cores through oracle/cref (C++/OpenMP restatement, kind
    "port"; the reference's own CPU path, onnxruntime + llama.cpp b7798, is not buildable here: SURVEY §8(c)):
    fp32 encoder + adaptor + CTC head on one 60 s clip, q8_0 prefill of 73 + 126 + 5 rows, 253 greedy decode
    steps (llama.cpp's ggml_vec_dot_q8_0_q8_0 arithmetic on AVX2). Weight synthesis is outside the timer."""
    from oracle import cref, synth
    from fun_asr_gguf.synthetic import synth_audio
    cores = cref.threads()
    enc = cref.CEncoder(synth.ENC_FULL)
    llm = cref.CQwen3(synth.LLM_FULL, n_ctx=512)
    a = synth_audio(int(CLIP_S * SR), 0)
    rng = np.random.default_rng(1234)
    t0 = time.perf_counter()
    r = enc.encode(a)
    t_enc = time.perf_counter() - t0
    prompt = np.concatenate([llm.embed_prompt(rng.integers(0, 151933, N_PREFIX)), r["audio_embd"],
                             llm.embed_prompt(rng.integers(0, 151933, N_SUFFIX))], 0)
    t1 = time.perf_counter()
    lg = llm.forward(prompt, 0)
    t_pre = time.perf_counter() - t1
    pos = prompt.shape[0]
    t2 = time.perf_counter()
    for _ in range(N_GEN):
        lg = llm.forward(llm.embed_tokens([int(np.argmax(lg))]), pos)
        pos += 1
    t_gen = time.perf_counter() - t2
    t_clip = time.perf_counter() - t0
    enc.close()
    llm.close()
    return {"value": round(CLIP_S / t_clip, 4), "unit": "audio_s/s", "cores": cores, "kind": "port",
            "sample": f"one full C2 clip, unextrapolated, oracle/cref C++/OpenMP on {cores} threads: 60 s fp32 "
                      f"encoder+adaptor+CTC {t_enc:.2f} s, q8_0 prefill 204 rows {t_pre:.2f} s, 253 greedy steps "
                      f"{t_gen:.2f} s ({t_gen / N_GEN * 1e3:.1f} ms/step); total {t_clip:.2f} s per 60 s clip "
                      f"(README.md:292-306 laptop CPU anchor: 7.19 s)"}


def pmc_mfma_busy(mode):
    """MFMA-pipe busy fraction per encoder kernel class from the committed counter pass of `mode` (scripts/pmc_mfma.py:
    SQ_VALU_MFMA_BUSY_CYCLES over the CUs' cycles while the class runs, rocprofv3 --pmc on bench.py itself), or {}."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*pmc_mfma_{mode}*.json")))
    if not files:
        return {}
    try:
        d = json.load(open(files[-1]))
        return {k: round(v["mfma_busy"], 4) for k, v in d.items() if isinstance(v, dict) and "mfma_busy" in v}, \
            os.path.basename(files[-1])
    except Exception:
        return {}


def pmc_traffic():
    """Per-launch HBM bytes of the decode-layer class from the committed PMC pass (scripts/pmc_traffic.py, rocprofv3
    --pmc FETCH_SIZE with the gfx950 x2 correction) taken with the batch-1 L2 prefetch slabs OFF (newest
    profiles/*pmc_gemv*slabs_off*.json, else the newest *pmc_gemv*.json): with the slabs on, the attention launch's
    pulls for the next two launches are counted in it while the consumers' reads are counted again (the counter pass
    brackets every dispatch, so the pulled lines do not survive to the consumer: its L2 hit rate is the same with and
    without the slabs, profiles/r05_pmc_l2hit_slabs_*.json). Returns (bytes, source, extra) or None."""
    import glob
    prof = os.path.join(ROOT, "profiles")
    files = sorted(glob.glob(os.path.join(prof, "*pmc_gemv*slabs_off*.json"))) or \
        sorted(glob.glob(os.path.join(prof, "*pmc_gemv*.json")))
    if not files:
        return None
    try:
        d = json.load(open(files[-1]))
        m = d["decode_layer_gemv_mean"]
        extra = {"traffic_over_weight_bytes": round(m["traffic_bytes"] / m["algorithmic_bytes"], 3)}
        on = sorted(glob.glob(os.path.join(prof, "*pmc_gemv*slabs_on*.json")))
        if on:
            extra["traffic_slabs_on"] = round(json.load(open(on[-1]))["decode_layer_gemv_mean"]["traffic_bytes"])
        for tag in ("off", "on"):
            hf = sorted(glob.glob(os.path.join(prof, f"*pmc_l2hit*slabs_{tag}*.json")))
            if hf:
                h = json.load(open(hf[-1]))
                extra[f"l2_hit_rate_slabs_{tag}"] = {k: round(v["hit_rate"], 3) for k, v in h.items()
                                                      if isinstance(v, dict) and "hit_rate" in v}
        return round(m["traffic_bytes"]), "profiles/" + os.path.basename(files[-1]), extra
    except Exception:
        return None


def graph_step_ms(engine, n_seq, steps=128, rows=204, seed=5):
    """Box-normalised decode figure: ms per graph-replayed decode step of n_seq sequences after a `rows`-row prefill
    each (n_past rows .. rows + steps + 4), the production step graphs, no profiling events."""
    rng = np.random.default_rng(seed)
    seqs = list(range(n_seq))
    for s in seqs:
        engine.llm_reset(s)
    E = engine.llm_cfg["n_embd"]
    engine.llm_prefill_batch(seqs, [(rng.standard_normal((rows, E)) * 0.05).astype(np.float32) for _ in seqs])
    engine.llm_generate(seqs, 4)
    engine.synchronize()
    t = time.perf_counter()
    engine.llm_generate(seqs, steps)
    engine.synchronize()
    return round((time.perf_counter() - t) / steps * 1e3, 4)


def c3_leg(batch, steps, warmup, device, model, barrier, dist):
    """configs[2] (C3): `batch` x 60 s clips per GPU per step, encoder batch + decoder continuous batch
    (prefill per sequence, then all sequences decode together: 253 greedy steps each, EOS ignored). Inputs
    resident in HBM. Returns whole-job audio_s/s (max-over-ranks time) and per-stage ms per step."""
    from fun_asr_gguf import FunASREngine
    from fun_asr_gguf.nano_dataclass import RecognitionStream
    from fun_asr_gguf.synthetic import synth_audio
    eng = FunASREngine("synthetic", "synthetic", "synthetic", "synthetic", n_predict=N_GEN, device=device,
                       model=model, ignore_eos=True, max_batch=batch, n_ctx=512)
    if not eng.initialize(verbose=False):
        raise RuntimeError("C3 engine init failed")
    m = eng.models
    rng = np.random.default_rng(1234)
    m.prompt_builder.fixed_ids = (list(rng.integers(0, m.llm_cfg["n_vocab"] - 3, N_PREFIX)),
                                  list(rng.integers(0, m.llm_cfg["n_vocab"] - 3, N_SUFFIX)))
    rank = dist.get_rank() if dist is not None else 0
    clips = [synth_audio(int(CLIP_S * SR), 1000 + rank * batch + i) for i in range(batch)]
    streams = []
    for c in clips:
        st = RecognitionStream()
        st.accept_waveform(SR, c)
        streams.append(st)
    handle = m.engine.upload(clips)
    dec = eng.orchestrator.decoder

    def step():
        rs = dec.decode_streams(streams, verbose=False, temperature=0.0, resident=handle)
        assert all(r.n_gen == N_GEN for r in rs), [r.n_gen for r in rs]
        return rs

    for _ in range(warmup):
        step()
    m.engine.synchronize()
    barrier()
    t0 = time.perf_counter()
    stage = np.zeros(6)
    for _ in range(steps):
        rs = step()
        tm = rs[0].timings
        # per-stream shares (ctc, prepare, inject, align are the batch's time / batch) -> the batch's time
        stage += [tm.encode, tm.ctc * batch, tm.prepare * batch, tm.inject * batch, tm.llm_generate, tm.align * batch]
    m.engine.synchronize()
    dt = time.perf_counter() - t0
    barrier()
    if dist is not None:
        import torch
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    world = dist.get_world_size() if dist is not None else 1
    step_ms = graph_step_ms(m.engine, batch)
    eng.cleanup()
    return {"workload": f"configs[2]: {batch} x 60 s clips per GPU per step (encoder batch {batch}, decoder continuous "
                        f"batch {batch}, 204-token prefill per clip, 253 greedy steps, EOS ignored)",
            "decode_step_ms_graph": step_ms,
            "decode_step_note": f"graph-replayed batch-{batch} decode step at n_past 208-335 (box-normalised decode figure)",
            "value": round(CLIP_S * batch * steps * world / dt, 2), "unit": "audio_s/s", "steps": steps,
            "warmup": warmup, "ms_per_step": round(dt / steps * 1e3, 2),
            "stage_ms": {k: round(v / steps * 1e3, 2) for k, v in zip(["encode", "ctc", "prompt", "prefill", "generate",
                                                                        "align"], stage)}}


def c3_varlen_leg(n_clips, batch, device, model, barrier, dist):
    """configs[2] with variable decode lengths: n_clips x 60 s clips on `batch` sequence slots, each clip's decode
    length pinned to a seeded draw from U[128, 384] tokens (mean 256 ~ the README's 253; stands in for EOS, which
    synthetic weights do not emit). Continuous batching (core/scheduler.py: a finished clip's slot is refilled with the
    next waiting clip, admitted as an encoder batch + prefill) against static groups of `batch` clips that each run
    to their longest member. The PCM goes host -> HBM inside the call (PCIe-inclusive)."""
    from fun_asr_gguf import FunASREngine
    from fun_asr_gguf.nano_dataclass import RecognitionStream
    from fun_asr_gguf.synthetic import synth_audio
    eng = FunASREngine("synthetic", "synthetic", "synthetic", "synthetic", n_predict=384, device=device,
                       model=model, ignore_eos=True, max_batch=batch, n_ctx=640)
    if not eng.initialize(verbose=False):
        raise RuntimeError("C3 varlen engine init failed")
    m = eng.models
    rng = np.random.default_rng(1234)
    m.prompt_builder.fixed_ids = (list(rng.integers(0, m.llm_cfg["n_vocab"] - 3, N_PREFIX)),
                                  list(rng.integers(0, m.llm_cfg["n_vocab"] - 3, N_SUFFIX)))
    rank = dist.get_rank() if dist is not None else 0
    clips = [synth_audio(int(CLIP_S * SR), 3000 + rank * n_clips + i) for i in range(n_clips)]
    lens = [int(x) for x in np.random.default_rng(77 + rank).integers(128, 385, n_clips)]
    orch = eng.orchestrator

    def continuous():
        return orch.decode_segments(clips, None, None, False, 0.0, 1.0, 50, n_predicts=lens)

    def static():
        out = []
        for i in range(0, n_clips, batch):
            sts = []
            for c in clips[i:i + batch]:
                st = RecognitionStream()
                st.accept_waveform(SR, c)
                sts.append(st)
            out += orch.decoder.decode_streams(sts, verbose=False, temperature=0.0, n_predicts=lens[i:i + batch])
        return out

    res = {}
    for name, fn in (("continuous", continuous), ("static", static)):
        rs = fn()  # warm-up (graphs for every batch width)
        assert [r.n_gen for r in rs] == lens
        m.engine.synchronize()
        barrier()
        t0 = time.perf_counter()
        fn()
        m.engine.synchronize()
        dt = time.perf_counter() - t0
        barrier()
        if dist is not None:
            import torch
            tt = torch.tensor([dt], dtype=torch.float64, device="cuda")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dt = float(tt.item())
        world = dist.get_world_size() if dist is not None else 1
        res[name] = {"value": round(CLIP_S * n_clips * world / dt, 2), "ms": round(dt * 1e3, 2)}
    st = orch.batcher.stats if hasattr(orch, "batcher") else {}
    eng.cleanup()
    return {"workload": f"configs[2] variable length: {n_clips} x 60 s clips per GPU on {batch} slots, decode lengths "
                        f"U[128, 384] (mean {np.mean(lens):.0f} tokens, pinned per clip)", "unit": "audio_s/s",
            "continuous": res["continuous"], "static": res["static"],
            "speedup": round(res["continuous"]["value"] / res["static"]["value"], 3),
            "scheduler": st}


# configs[4]'s hotword/context prompt: the reference's prompt text (prompt_utils.py:16-54) for this context and hotword
# list, tokenized by the product's GGUF tokenizer (fa_tokenize) with the repo's synthetic Qwen2 BPE vocabulary (no
# real tokenizer ships in this image): 73 prefix + 5 suffix tokens, the lengths configs[4] names
C5_CONTEXT = "这是一段关于人工智能的会议"
C5_HOTWORDS = ["通义千问", "语音识别", "魔搭社区", "大模型"]


def c5_prompt_ids():
    from fun_asr_gguf._native import Vocab
    from fun_asr_gguf.prompt_utils import prompt_texts
    v = Vocab(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden", "tokenizer_qwen2_synth.gguf"))
    p, s = prompt_texts(C5_HOTWORDS, None, C5_CONTEXT)
    pi, si = v.tokenize(p), v.tokenize(s)
    assert (len(pi), len(si)) == (N_PREFIX, N_SUFFIX), (len(pi), len(si))
    return list(pi), list(si)


def c4_leg(steps, warmup, device, model, barrier, dist):
    """configs[3] (C4): one 300 s file, segment_size 60 / overlap 4 -> 6 segments {0-60, 56-116, ..., 280-300}
    (orchestrator.py:123-136) through the public FunASREngine.transcribe long path. N=1: all segments as one
    device batch. N>1: segments assigned longest-first to ranks (fun_asr_gguf.parallel), records gathered to
    rank 0 through the engine's own RCCL communicator (fa_comm_allgather_*), merged there. Every segment decodes 253 greedy tokens, EOS ignored (the
    20 s segment too, above its pinned 85: conservative). The PCM goes host -> HBM inside the call (PCIe-inclusive)."""
    from fun_asr_gguf import FunASREngine
    from fun_asr_gguf.synthetic import synth_audio
    eng = FunASREngine("synthetic", "synthetic", "synthetic", "synthetic", n_predict=N_GEN, device=device,
                       model=model, ignore_eos=True, max_batch=6, n_ctx=512)
    if not eng.initialize(verbose=False):
        raise RuntimeError("C4 engine init failed")
    m = eng.models
    rng = np.random.default_rng(1234)
    m.prompt_builder.fixed_ids = (list(rng.integers(0, m.llm_cfg["n_vocab"] - 3, N_PREFIX)),
                                  list(rng.integers(0, m.llm_cfg["n_vocab"] - 3, N_SUFFIX)))
    audio = synth_audio(300 * SR, 4000)
    if dist is not None:  # the records gather to rank 0 through the engine's own RCCL communicator (fa_comm_*)
        from fun_asr_gguf.parallel import init_native_comm
        init_native_comm(m.engine, dist)

    def step():
        return eng.transcribe(audio, segment_size=60.0, overlap=4.0, temperature=0.0, verbose=False, ranks=dist)

    for _ in range(warmup):
        r = step()
    m.engine.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        r = step()
    m.engine.synchronize()
    dt = time.perf_counter() - t0
    barrier()
    if dist is not None:
        import torch
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    world = dist.get_world_size() if dist is not None else 1
    n_chars = len(r.segments) if r is not None and r.segments else 0
    eng.cleanup()
    return {"workload": "configs[3]: one 300 s file, segment 60 / overlap 4 (6 segments), public transcribe() long "
                        f"path, {'one device batch' if world == 1 else f'LPT-sharded over {world} ranks + gather to rank 0'}"
                        ", 253 greedy steps per segment, EOS ignored, merge on rank 0",
            "value": round(300.0 * steps / dt, 2), "unit": "audio_s/s (whole job, one file)", "steps": steps,
            "warmup": warmup, "ms_per_step": round(dt / steps * 1e3, 2), "rtf": round(dt / steps / 300.0, 6),
            "merged_chars": n_chars}


def c5_long_leg(steps, warmup, device, model, barrier, dist):
    """configs[4] as configs[3]'s long-audio path: the 300 s file (6 segments of 60 s / overlap 4) with the fp16 encoder
    graph (02-Quantize-ONNX.py:13-27) and the 73-token hotword/context prefix (C5_CONTEXT / C5_HOTWORDS through the
    GGUF tokenizer) on every segment, through transcribe(); N>1: segment-parallel (LPT over the ranks, records gathered
    through the engine's RCCL communicator). 253 greedy steps per segment, EOS ignored."""
    from fun_asr_gguf import FunASREngine
    from fun_asr_gguf.synthetic import synth_audio
    eng = FunASREngine("synthetic", "synthetic", "synthetic", "synthetic", n_predict=N_GEN, device=device,
                       model=model, ignore_eos=True, max_batch=6, n_ctx=512)
    if not eng.initialize(verbose=False):
        raise RuntimeError("C5 engine init failed")
    m = eng.models
    m.engine.set_encoder_fp16(True)
    m.prompt_builder.fixed_ids = c5_prompt_ids()
    audio = synth_audio(300 * SR, 4000)
    if dist is not None:
        from fun_asr_gguf.parallel import init_native_comm
        init_native_comm(m.engine, dist)

    def step():
        return eng.transcribe(audio, segment_size=60.0, overlap=4.0, temperature=0.0, verbose=False, ranks=dist)

    for _ in range(warmup):
        step()
    m.engine.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        r = step()
    m.engine.synchronize()
    dt = time.perf_counter() - t0
    barrier()
    if dist is not None:
        import torch
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    world = dist.get_world_size() if dist is not None else 1
    eng.cleanup()
    return {"workload": "configs[4]: the 300 s file (6 segments), fp16 encoder graph + q8_0 LLM, 73-token hotword/context "
                        f"prefix on every segment, {'one device batch' if world == 1 else f'segment-parallel over {world} ranks'}"
                        ", 253 greedy steps per segment, EOS ignored",
            "value": round(300.0 * steps / dt, 2), "unit": "audio_s/s (whole job, one file)", "steps": steps,
            "ms_per_step": round(dt / steps * 1e3, 2), "rtf": round(dt / steps / 300.0, 6)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= ranks) of the job; without WORLD_SIZE in the environment, N > 1 spawns N ranks")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--model", default="full")
    ap.add_argument("--c3-batch", type=int, default=32, help="clips per step of the C3 leg (0 = skip)")
    ap.add_argument("--c3-steps", type=int, default=2)
    ap.add_argument("--c4-steps", type=int, default=2)
    ap.add_argument("--c3-varlen", type=int, default=192, help="clips of the variable-length C3 leg (0 = skip)")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 (300 s long-audio) leg")
    ap.add_argument("--c2-only", action="store_true",
                    help="the headline leg alone (counter-collection runs, where every dispatch is serialised)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        # no launcher: become one: N fresh rank processes, started before this process touches a GPU
        rc, text = spawn_ranks(args.gpus, sys.argv[1:])
        if text:
            sys.stdout.write(text)
            sys.stdout.flush()
        sys.exit(rc if 0 <= rc < 256 else 128 + (-rc if rc < 0 else 1))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    args.launcher = os.environ.get("BENCH_LAUNCHER", "torchrun" if world > 1 else "single")
    dist = None
    # BENCH_FORCE_DIST=1: the multi-rank code path (RCCL process group, barriers, max-over-ranks timing, sharded
    # transcribe with the engine-native gather) at world size 1 -- a one-GPU rehearsal of what N > 1 runs
    if world > 1 or os.environ.get("BENCH_FORCE_DIST") == "1":
        import torch
        import torch.distributed as tdist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dist = tdist
        assert dist.get_world_size() == world, (dist.get_world_size(), world)

    def barrier():
        if dist is not None:
            dist.barrier()

    from fun_asr_gguf import FunASREngine
    from fun_asr_gguf.nano_dataclass import RecognitionStream
    from fun_asr_gguf.synthetic import synth_audio

    eng = FunASREngine("synthetic", "synthetic", "synthetic", "synthetic", n_predict=N_GEN, device=local,
                       model=args.model, ignore_eos=True)
    if not eng.initialize(verbose=False):
        raise RuntimeError("engine init failed")
    m = eng.models
    rng = np.random.default_rng(1234)
    m.prompt_builder.fixed_ids = (list(rng.integers(0, m.llm_cfg["n_vocab"] - 3, N_PREFIX)),
                                  list(rng.integers(0, m.llm_cfg["n_vocab"] - 3, N_SUFFIX)))
    clip = synth_audio(int(CLIP_S * SR), rank)
    st = RecognitionStream()
    st.accept_waveform(SR, clip)
    handle = m.engine.upload([clip])
    dec = eng.orchestrator.decoder

    def step():
        return dec.decode_streams([st], verbose=False, temperature=0.0, resident=handle)[0]

    for _ in range(args.warmup):
        res = step()
        assert res.n_gen == N_GEN, res.n_gen
    m.engine.synchronize()
    log("[bench] C2 warmup done")
    barrier()
    # ---- timed region (production path: hipGraph decode steps, no timing events)
    t0 = time.perf_counter()
    stage = np.zeros(6)
    for _ in range(args.steps):
        res = step()
        tm = res.timings
        stage += [tm.encode, tm.ctc, tm.prepare, tm.inject, tm.llm_generate, tm.align]
    m.engine.synchronize()
    dt = time.perf_counter() - t0
    log("[bench] C2 timed steps done")
    barrier()
    # ---- roofline pass: same steps with HIP events on the engine stream around every launch of each
    # kernel class (decode: event nodes captured inside the step graph, replayed on the last step of every
    # 32-step chunk, i.e. a uniform sample of the decode launches)
    m.engine.profile_enable(True)
    tp = time.perf_counter()
    for _ in range(args.steps):
        step()
    m.engine.synchronize()
    dt_prof = time.perf_counter() - tp
    prof = {c: m.engine.profile_read(c) for c in range(7)}
    m.engine.profile_enable(False)
    step1_ms = graph_step_ms(m.engine, 1)
    barrier()
    if dist is not None:
        import torch
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    out = {}
    if rank == 0:
        out = headline(args, world, dt, dt_prof, prof, stage)
        out["decode_step_ms_graph"] = step1_ms  # graph-replayed batch-1 step at n_past 208-335 (box-normalised)
    log("[bench] C2 headline leg done")
    if args.c2_only:
        eng.cleanup()
        if rank == 0:
            print(json.dumps(out, ensure_ascii=False), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return
    # ---- C5 leg (configs[4] on one GPU): the same clip with the fp16 encoder graph (02-Quantize-ONNX.py) and the
    # 73-token prefix; the 8-GPU segment-parallel part is the driver's scaling run of the same entry point
    m.engine.set_encoder_fp16(True)
    fixed = m.prompt_builder.fixed_ids
    m.prompt_builder.fixed_ids = c5_prompt_ids()
    step()
    m.engine.synchronize()
    barrier()
    t5 = time.perf_counter()
    st5 = np.zeros(6)
    for _ in range(args.steps):
        tm = step().timings
        st5 += [tm.encode, tm.ctc, tm.prepare, tm.inject, tm.llm_generate, tm.align]
    m.engine.synchronize()
    dt5 = time.perf_counter() - t5
    m.engine.set_encoder_fp16(False)
    m.prompt_builder.fixed_ids = fixed
    # secondary leg: the default transcribe() sampling (temperature 0.4, top_k 50 -> top_p 1.0 -> temp -> dist on
    # device, asr_engine.py:65), same clip and pinned length
    step_s = lambda: dec.decode_streams([st], verbose=False, temperature=0.4, top_k=50, resident=handle)[0]
    step_s()
    m.engine.synchronize()
    ts = time.perf_counter()
    gen_s = 0.0
    for _ in range(args.steps):
        r_s = step_s()
        assert r_s.n_gen == N_GEN, r_s.n_gen
        gen_s += r_s.timings.llm_generate
    m.engine.synchronize()
    dts = time.perf_counter() - ts
    if rank == 0:
        out["c2_sampled"] = {"workload": "configs[1] clip with the default sampler chain (temperature 0.4, top_k 50)",
                             "value": round(CLIP_S * args.steps / dts, 3), "unit": "audio_s/s",
                             "ms_per_step": round(dts / args.steps * 1e3, 3),
                             "generate_ms": round(gen_s / args.steps * 1e3, 3)}
    # exact-f32 leg: the same clip with the encoder GEMMs and attention on v_mfma_f32_32x32x2_f32 (fa_set_encoder_gemm(0),
    # the reference graph's arithmetic without the bf16x3 operand split)
    m.engine.set_encoder_gemm("f32")
    step()
    m.engine.synchronize()
    barrier()
    tf = time.perf_counter()
    stf = np.zeros(6)
    for _ in range(args.steps):
        tm = step().timings
        stf += [tm.encode, tm.ctc, tm.prepare, tm.inject, tm.llm_generate, tm.align]
    m.engine.synchronize()
    dtf = time.perf_counter() - tf
    m.engine.set_encoder_gemm("bf16x3")
    if rank == 0:
        out["c2_exact_f32"] = {"workload": "configs[1] clip with exact-f32 MFMA encoder GEMMs / attention "
                                           "(fa_set_encoder_gemm(0))",
                               "value": round(CLIP_S * args.steps / dtf, 3), "unit": "audio_s/s",
                               "ms_per_step": round(dtf / args.steps * 1e3, 3),
                               "stage_ms": {k: round(v / args.steps * 1e3, 3) for k, v in zip(
                                   ["encode", "ctc", "prompt", "prefill", "generate", "align"], stf)}}
    if rank == 0:
        out["c5"] = {"workload": "configs[4] on 1 GPU: single 60 s clip, fp16 encoder graph + q8_0 LLM, 73-token "
                                 "context + hotword prefix (prompt_texts(C5_HOTWORDS, context=C5_CONTEXT) through the "
                                 "GGUF tokenizer of tests/golden/tokenizer_qwen2_synth.gguf)",
                     "value": round(CLIP_S * args.steps / dt5, 3), "unit": "audio_s/s",
                     "ms_per_step": round(dt5 / args.steps * 1e3, 3),
                     "stage_ms": {k: round(v / args.steps * 1e3, 3) for k, v in zip(
                         ["encode", "ctc", "prompt", "prefill", "generate", "align"], st5)}}
    eng.cleanup()
    log("[bench] C5 / sampled / exact-f32 legs done")
    if args.c3_batch > 0:
        try:
            out["c3"] = c3_leg(args.c3_batch, args.c3_steps, 1, local, args.model, barrier, dist)
        except Exception as e:  # reported, never fatal for the headline number
            out["c3"] = {"value": None, "error": str(e)[:300]}
        log("[bench] C3 leg done")
    if args.c3_varlen > 0:
        try:
            out["c3_varlen"] = c3_varlen_leg(args.c3_varlen, args.c3_batch or 32, local, args.model, barrier, dist)
        except Exception as e:  # reported, never fatal for the headline number
            out["c3_varlen"] = {"value": None, "error": str(e)[:300]}
        log("[bench] C3 varlen leg done")
    if not args.no_c4:
        try:
            out["c4"] = c4_leg(args.c4_steps, 1, local, args.model, barrier, dist)
        except Exception as e:  # reported, never fatal for the headline number
            out["c4"] = {"value": None, "error": str(e)[:300]}
        log("[bench] C4 leg done")
        try:
            out["c5_long"] = c5_long_leg(args.c4_steps, 1, local, args.model, barrier, dist)
        except Exception as e:  # reported, never fatal for the headline number
            out["c5_long"] = {"value": None, "error": str(e)[:300]}
    if rank == 0:
        print(json.dumps(out, ensure_ascii=False), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def headline(args, world, dt, dt_prof, prof, stage):
    audio_s = CLIP_S * args.steps * world
    value = audio_s / dt
    ms_step = dt / args.steps * 1e3
    # dominant kernel class by estimated device time: decoder layer classes are timed on layers 0 and 1 only
    # (identical shapes in all layers): layer 1 (L2-warm weights from the prefetch slabs, as in every layer but 0)
    # stands for layers 1 .. n_layer - 1, layer 0 is its own class (5); prefill forwards are class 6
    bf3 = os.environ.get("FUNASR_ENC_GEMM", "bf16x3") != "f32"
    enc_peak = BF16X3_PEAK_TFS if bf3 else FP32_MFMA_PEAK_TFS
    names = {0: "q8_0 GEMV/GEMM (decoder layers)",
             1: "bf16x3 MFMA GEMM (f32 encoder)" if bf3 else "f32 MFMA GEMM (encoder)",
             2: "bf16x3 MFMA attention (f32 encoder)" if bf3 else "f32 MFMA attention (encoder)",
             3: "decode attention", 4: "q8_0 LM head GEMV + argmax", 6: "prefill layer launches (sampled layers)"}
    n_layer = 28 if args.model == "full" else 2
    prof = dict(prof)
    l0 = prof.pop(5)
    if n_layer > 2 and l0["launches"]:  # decode layers: layer 0 + (n_layer - 1) x layer 1 (class 0 holds layer 1)
        p0 = prof[0]
        prof[0] = {k: p0[k] * (n_layer - 1) + l0[k] for k in ("ms", "bytes", "flops", "launches")}
        layer_note = {"layer0_avg_launch_us": round(l0["ms"] * 1e3 / l0["launches"], 2),
                      "layer1_avg_launch_us": round(p0["ms"] * 1e3 / max(1, p0["launches"]), 2)}
        weight = {0: 1, 1: 1, 2: 1, 3: n_layer, 4: 1, 6: n_layer / 2}
    else:
        layer_note = {}
        weight = {0: n_layer, 1: 1, 2: 1, 3: n_layer, 4: 1, 6: n_layer}
    est_ms = {c: prof[c]["ms"] * weight[c] for c in prof}
    dom = max(prof, key=lambda c: est_ms[c])
    p = prof[dom]
    avg_s = p["ms"] / max(1, p["launches"]) / 1e3
    if dom in (0, 4):
        ach = p["bytes"] / max(1, p["launches"]) / avg_s / 1e9
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None}
        pt = pmc_traffic() if dom == 0 else None
        if pt:
            roof["traffic"] = pt[0]
            roof["traffic_source"] = pt[1]
            roof.update(pt[2])
    else:
        ach = p["flops"] / max(1, p["launches"]) / avg_s / 1e12
        roof = {"bound": "mfma", "achieved": round(ach, 2), "peak": round(enc_peak, 1), "unit": "TFLOP/s",
                "frac": round(ach / enc_peak, 4), "traffic": None}
    if dom == 0:
        roof.update(layer_note)
    roof.update(kernel=names[dom], avg_launch_us=round(avg_s * 1e6, 2), launches_timed=round(p["launches"]),
                per_launch=("q8_0 weight bytes (+ the two-launch layer's K/V rows)" if dom == 0 else
                            "q8_0 weight bytes" if dom == 4 else "algorithmic FLOPs"),
                est_device_ms_per_step={names[c]: round(est_ms[c] / args.steps, 2) for c in prof})
    if dom == 0 and roof.get("traffic"):
        roof["traffic_note"] = ("FETCH_SIZE x 2 per decode-layer launch (mean of the attention and FFN launches), graph "
                                "path, batch-1 L2 prefetch slabs off: the HBM bytes the launches need (weights, K/V rows, "
                                "activations). With the slabs on the counter pass also counts the attention launch's "
                                "pulls for the next two launches (traffic_slabs_on), which the bracketed dispatches of "
                                "a counter pass do not keep for the consumers (same FFN-launch L2 hit rate either way); "
                                "DESIGN.md section 3")
    # the encoder's MFMA classes (secondary: the clip's 705 GFLOP of f32 contractions) against the peak of the
    # arithmetic they run on: bf16x3 = three bf16 MFMA products per f32 product (2.5 PF/s / 3), or exact f32
    for c, key in ((1, "encoder_gemm"), (2, "encoder_attention")):
        e = prof[c]
        if e["launches"] and e["ms"] > 0:
            tfs = e["flops"] / (e["ms"] / 1e3) / 1e12
            roof[key] = {"achieved_TFs": round(tfs, 2), "peak_TFs": round(enc_peak, 1), "arith": "bf16x3" if bf3 else "f32",
                         "frac": round(tfs / enc_peak, 4), "avg_launch_us": round(e["ms"] * 1e3 / e["launches"], 2)}
            busy = pmc_mfma_busy("bf16x3" if bf3 else "f32")
            if busy:
                cls = {"encoder_gemm": "encoder GEMM (bf16x3)" if bf3 else "encoder GEMM (exact f32 / STFT / mel)",
                       "encoder_attention": "encoder attention (bf16x3)" if bf3 else "encoder attention (exact f32)"}[key]
                if cls in busy[0]:  # counter-derived MFMA utilisation (the batch-32 encode of the PMC pass)
                    roof[key]["mfma_busy"] = busy[0][cls]
                    roof[key]["mfma_busy_source"] = "profiles/" + busy[1]
    lm = prof[4]
    if lm["launches"]:
        lm_s = lm["ms"] / lm["launches"] / 1e3
        roof["lm_head"] = {"achieved_GBs": round(lm["bytes"] / lm["launches"] / lm_s / 1e9, 1),
                           "avg_launch_us": round(lm_s * 1e6, 2)}
    out = {"metric": "audio-sec/s (RTF = 1/value per GPU) on 60 s 16 kHz clips", "value": round(value, 3),
           "unit": "audio_s/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "f32 encoder (bf16x3 split-operand MFMA GEMMs, f32 accumulate) / q8_0 x q8_0 int-dot decoder", "data": "synthetic (seeded chirps; synthetic weights)",
           "rtf": round(1.0 / (value / world), 6),
           "config": {"workload": "configs[1]: single 60 s clip per GPU per step, fp32 encoder + CTC + q8_0 LLM "
                                  "(73+126+5 prefill, 253 greedy steps, EOS ignored)",
                      "model": "Fun-ASR-Nano (SenseVoiceSmall enc 70 SANM blocks + Qwen3-0.6B q8_0)",
                      "global_batch": world, "seq_len": int(CLIP_S * SR), "parallelism": f"dp{world}",
                      "ranks": world, "launcher": args.launcher,
                      "gpus_flag": args.gpus if args.gpus is not None else world},
           "stage_ms": {k: round(v / args.steps * 1e3, 3) for k, v in zip(
               ["encode", "ctc", "prompt", "prefill", "generate", "align"], stage)},
           "profiled_pass_ms_per_step": round(dt_prof / args.steps * 1e3, 3),
           "kernel_class_avg_us": {names[c]: round(prof[c]["ms"] * 1e3 / max(1, prof[c]["launches"]), 2) for c in prof},
           "roofline": roof}
    if not args.no_cpu_baseline and world == 1:  # on rank 0 at N = 1 only
        try:
            out["cpu_baseline"] = cpu_baseline()
        except Exception as e:  # reported, never fatal for the GPU number
            out["cpu_baseline"] = {"value": None, "error": str(e)[:200]}
    return out


if __name__ == "__main__":
    main()
