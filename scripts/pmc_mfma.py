"""MFMA utilisation of the encoder's matrix kernels from a rocprofv3 PMC pass on bench.py
(`--pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE`, scripts/gpu_pmc_mfma.sh).

Counter semantics (MI355X_MICROARCH.md, per-instruction table and DVFS note): SQ_VALU_MFMA_BUSY_CYCLES sums the cycles
the SIMDs' matrix pipes are busy (32 per v_mfma_f32_32x32x16_bf16); GRBM_GUI_ACTIVE sums the busy cycles of the 8
XCDs. mfma_busy = MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) is the fraction of the chip's matrix-pipe cycles the
kernel kept busy while it ran (a bf16 dense-peak fraction for bf16 / bf16x3 MFMAs; for v_mfma_f32_32x32x2_f32, which
runs at 1/16 of the bf16 rate, busy cycles count the same pipe and the fraction is the f32-pipe utilisation).
Usage: python scripts/pmc_mfma.py <results.db> <out.json>
"""
import json
import sqlite3
import sys
from collections import defaultdict

CLASSES = {  # kernel-name substring -> class (first match; the fp16 graph's P = 1 instances of the bf16x3 family first)
    "PrecB<1>": "encoder GEMM (fp16 graph)",
    "k_attn_bf3<128, 1": "encoder attention (fp16 graph)",
    "k_attn_bf3<64, 1": "encoder attention (fp16 graph)",
    "k_gemm_bf3": "encoder GEMM (bf16x3)",
    "k_attn_bf3": "encoder attention (bf16x3)",
    "k_gemm_f32": "encoder GEMM (exact f32 / STFT / mel)",
    "k_attn_f32": "encoder attention (exact f32)",
    "k_gemm_f16": "encoder GEMM (fp16 graph)",
    "k_gemm_q8_t": "prefill q8_0 GEMM (tiled)",
    "k_gemm_q8_kw": "prefill q8_0 GEMM",
    "k_attn_prefill": "prefill attention",
}
N_SIMD = 256 * 4


def main():
    db, out = sys.argv[1], sys.argv[2]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(pmc_events)").fetchall()]
    disp = "dispatch_id" if "dispatch_id" in cols else ("correlation_id" if "correlation_id" in cols else None)
    sel = f"select name, counter_name, counter_value{', ' + disp if disp else ''} from pmc_events"
    per = defaultdict(lambda: defaultdict(float))
    launches = defaultdict(set)
    for row in c.execute(sel).fetchall():
        name, cn, val = row[0], row[1], float(row[2])
        for key, cls in CLASSES.items():
            if key in name:
                per[cls][cn] += val
                if disp:
                    launches[cls].add(row[3])
                break
    res = {}
    for cls, v in per.items():
        busy, grbm = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0), v.get("GRBM_GUI_ACTIVE", 0.0)
        res[cls] = {"launches": len(launches[cls]) or None, "SQ_VALU_MFMA_BUSY_CYCLES": busy,
                    "GRBM_GUI_ACTIVE": grbm, "SQ_BUSY_CU_CYCLES": v.get("SQ_BUSY_CU_CYCLES", 0.0),
                    "kernel_cycles": grbm / 8.0,
                    "mfma_busy": busy / (grbm / 8.0 * N_SIMD) if grbm > 0 else None}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
