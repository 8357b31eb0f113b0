#!/usr/bin/env python
"""Summarise a rocprofv3 kernel trace (kernel_trace.csv or results .db): per-dispatch durations of the LAST training step."""
import csv
import sys
from collections import defaultdict

def load(path):
    """kernel_trace.csv, or a rocprofv3 results .db (default output format)"""
    if path.endswith(".db"):
        import sqlite3
        c = sqlite3.connect(path)
        q = ("select name, start, end, grid_x, lds_size, vgpr_count, accum_vgpr_count, stream_id "
             "from kernels order by start")
        keys = ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "LDS_Block_Size",
                "VGPR_Count", "Accum_VGPR_Count", "Stream_Id"]
        return [dict(zip(keys, r)) for r in c.execute(q)]
    return list(csv.DictReader(open(path)))


rows = load(sys.argv[1])
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
# find adam dispatches as step boundaries
idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
if len(idx) >= 2:
    lo, hi = idx[-2] + 1, idx[-1] + 1
else:
    lo, hi = 0, len(rows)
tot = 0
agg = defaultdict(float)
for r in rows[lo:hi]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    name = r["Kernel_Name"]
    short = name.replace("void ", "").replace("ddlpc::(anonymous namespace)::", "")
    short = short.split("(")[0] if not short.startswith("(") else short
    short = short[:60]
    agg[short] += d
    if len(sys.argv) > 3:
        print(f"{d:9.1f}us grid={r['Grid_Size_X']:>9} lds={r['LDS_Block_Size']:>6} vgpr={r['VGPR_Count']}/{r['Accum_VGPR_Count']} {short}")
print(f"step span kernels: {hi - lo}, busy {tot / 1e3:.3f} ms, wall {(int(rows[hi-1]['End_Timestamp']) - int(rows[lo]['Start_Timestamp'])) / 1e6:.3f} ms")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:25]:
    print(f"{v:10.1f}us  {k}")
