"""Per-kernel L2 hit rate from a rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum pass (MI355X_MICROARCH.md §L2:
hit rate = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)), for the batch-1 decode launches (k_attn_o<true> = AB,
k_ffn_fused<1> = C) and the LM head, plus every other kernel with at least `min_launches` dispatches.
Usage: python scripts/pmc_l2hit.py <results.db> <out.json> [label]
"""
import json
import sqlite3
import sys
from collections import defaultdict

KEYS = {"k_attn_o<true>": "AB (q|k|v GEMV + attention + o slice)", "k_ffn_fused<1>": "C (gate|up + down slice)",
        "k_gemv_q8<1, 1, true, 3, true>": "LM head (batch 1)"}


def main():
    db, out = sys.argv[1], sys.argv[2]
    label = sys.argv[3] if len(sys.argv) > 3 else ""
    c = sqlite3.connect(db)
    rows = c.execute("select name, counter_value, counter_name from pmc_events").fetchall()
    agg = defaultdict(lambda: defaultdict(list))
    for name, val, cn in rows:
        for key in KEYS:
            if key in name:
                agg[key][cn].append(float(val))
    res = {"label": label}
    for key, cs in agg.items():
        hit, miss = cs.get("TCC_HIT_sum", []), cs.get("TCC_MISS_sum", [])
        if not hit or not miss:
            continue
        h, m = sum(hit) / len(hit), sum(miss) / len(miss)
        res[key] = {"what": KEYS[key], "launches": len(hit), "tcc_hit_mean": h, "tcc_miss_mean": m,
                    "hit_rate": h / max(1.0, h + m)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
