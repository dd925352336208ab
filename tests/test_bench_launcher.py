"""bench.py's own rank launcher (`python bench.py --gpus N` with no WORLD_SIZE in the environment): N fresh rank
processes with torchrun's environment, started by a parent that imports no torch and touches no GPU; rank 0's stdout
is the job's line; a failing rank ends the job with a nonzero code instead of leaving its peers blocked."""
import json
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUB = textwrap.dedent("""
    import json, os, sys, time
    out = os.environ["STUB_OUT"]
    keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "BENCH_LAUNCHER"]
    rec = {k: os.environ.get(k) for k in keys}
    rec.update(pid=os.getpid(), ppid=os.getppid(), argv=sys.argv[1:])
    with open(os.path.join(out, "rank%s.json" % os.environ["RANK"]), "w") as f:
        json.dump(rec, f)
    if os.environ.get("STUB_FAIL_RANK") == os.environ["RANK"]:
        sys.exit(3)
    if os.environ.get("STUB_FAIL_RANK") is not None:
        time.sleep(600)  # a peer blocked in a collective
    if os.environ["RANK"] == "0":
        print(json.dumps({"metric": "stub", "n_gpus": int(os.environ["WORLD_SIZE"])}))
""")

DRIVER = textwrap.dedent("""
    import json, sys
    sys.path.insert(0, {root!r})
    import bench
    rc, text = bench.spawn_ranks({n}, ["--steps", "1"], script={stub!r}, grace_s=1.0)
    print(json.dumps({{"rc": rc, "text": text, "torch_imported": "torch" in sys.modules,
                       "hip_loaded": any("amdhip" in l or "libfunasr_hip" in l for l in open("/proc/self/maps"))}}))
""")


def _run(tmp_path, n, fail_rank=None):
    stub = tmp_path / "stub.py"
    stub.write_text(STUB)
    env = dict(os.environ, STUB_OUT=str(tmp_path))
    env.pop("WORLD_SIZE", None)
    if fail_rank is not None:
        env["STUB_FAIL_RANK"] = str(fail_rank)
    r = subprocess.run([sys.executable, "-c", DRIVER.format(root=ROOT, n=n, stub=str(stub))], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_spawn_starts_n_distinct_ranks_without_gpu_in_parent(tmp_path):
    got = _run(tmp_path, 4)
    assert got["rc"] == 0
    assert not got["torch_imported"] and not got["hip_loaded"]
    assert json.loads(got["text"]) == {"metric": "stub", "n_gpus": 4}
    recs = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(4)]
    assert sorted(int(x["RANK"]) for x in recs) == [0, 1, 2, 3]
    assert [x["LOCAL_RANK"] for x in recs] == ["0", "1", "2", "3"]
    assert {x["WORLD_SIZE"] for x in recs} == {"4"} and {x["LOCAL_WORLD_SIZE"] for x in recs} == {"4"}
    assert {x["MASTER_ADDR"] for x in recs} == {"127.0.0.1"} and len({x["MASTER_PORT"] for x in recs}) == 1
    assert {x["BENCH_LAUNCHER"] for x in recs} == {"spawn"}
    assert len({x["pid"] for x in recs}) == 4 and len({x["ppid"] for x in recs}) == 1  # 4 children of one parent
    assert all(x["argv"] == ["--steps", "1"] for x in recs)


def test_failing_rank_ends_the_job(tmp_path):
    got = _run(tmp_path, 3, fail_rank=1)
    assert got["rc"] != 0  # rank 1 exited 3; ranks 0 and 2 (blocked) were killed after the grace period


def test_bench_module_imports_no_torch():
    r = subprocess.run([sys.executable, "-c", f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
                        "print('torch' in sys.modules)"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "False", r.stderr


def test_roofline_traffic_from_the_slabs_off_counter_pass():
    """roofline.traffic is FETCH_SIZE x 2 per decode-layer launch from the committed slabs-off pass, with the slabs-on
    traffic and the per-launch L2 hit rates of both passes beside it (profiles/r05_pmc_*)."""
    sys.path.insert(0, ROOT)
    import bench
    got = bench.pmc_traffic()
    assert got is not None
    traffic, src, extra = got
    assert "slabs_off" in src
    d = json.load(open(os.path.join(ROOT, src)))["decode_layer_gemv_mean"]
    assert traffic == round(d["traffic_bytes"]) and 1.0 < extra["traffic_over_weight_bytes"] < 1.3
    assert extra["traffic_slabs_on"] > traffic
    assert set(extra["l2_hit_rate_slabs_off"]) == set(extra["l2_hit_rate_slabs_on"]) == {"k_attn_o<true>", "k_ffn_fused<1>"}
