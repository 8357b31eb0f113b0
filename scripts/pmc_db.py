#!/usr/bin/env python
"""Per-kernel PMC summary of a rocprofv3 results database (``-d DIR -o run`` writes
DIR/run_results.db): the median over dispatches of every counter, plus the per-wave ratios
(WAIT_INST_ANY / WAVE_CYCLES, ACTIVE_INST_ANY / WAVE_CYCLES) when those counters are present.

    python scripts/pmc_db.py gpurun_out/gNN/pmc/run_results.db [kernel-name filter]
"""
import collections
import sqlite3
import statistics
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in c.execute("select * from counters_collection"):
        d = dict(zip(cols, r))
        name = d["kernel_name"].replace("void ", "").replace("ddlpc::(anonymous namespace)::", "")
        name = name.split("(")[0][:48]
        if filt and filt not in name:
            continue
        agg[name][d["counter_name"]].append(d["value"])
    for name, cs in sorted(agg.items()):
        med = {k: statistics.median(v) for k, v in cs.items()}
        extra = ""
        wc = med.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS"):
                if k in med:
                    extra += f" {k[8:]}/wave={med[k] / wc:.3f}"
        print(f"{name:48s} n={len(next(iter(cs.values())))} " +
              " ".join(f"{k}={v:.4g}" for k, v in sorted(med.items())) + extra)


if __name__ == "__main__":
    main()
