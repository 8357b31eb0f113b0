#!/usr/bin/env python
"""Per-queue busy time and per-phase (forward / backward) category totals of the last
training step in a rocprofv3 kernel_trace.csv (step = between the last two Adam launches)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
lo, hi = (idx[-2] + 1, idx[-1] + 1) if len(idx) >= 2 else (0, len(rows))
seg = rows[lo:hi]


def cat(n):
    for k in ("wgrad", "conv3_res", "conv3_fwd", "bn_bwd", "bn_relu", "bn_stats", "bn_grad",
              "gemm", "rows_", "head_", "splitk", "adam", "pack"):
        if k in n:
            return k
    return "other"


busy = defaultdict(float)
span = {}
for r in seg:
    q = r["Queue_Id"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy[q] += (e - s) / 1e3
    a, b = span.get(q, (s, e))
    span[q] = (min(a, s), max(b, e))
print("queues busy us:", {k: round(v) for k, v in busy.items()},
      "span us:", {k: round((b - a) / 1e3) for k, (a, b) in span.items()})
hb = next((i for i, r in enumerate(seg) if "head_ce_bwd" in r["Kernel_Name"]), len(seg))
t0 = int(seg[0]["Start_Timestamp"])
tb = int(seg[hb]["Start_Timestamp"]) if hb < len(seg) else t0
te = max(int(r["End_Timestamp"]) for r in seg)
print(f"forward wall {(tb - t0) / 1e6:.3f} ms, backward+optimizer wall {(te - tb) / 1e6:.3f} ms")
for name, part in (("fwd", seg[:hb]), ("bwd", seg[hb:])):
    c = defaultdict(lambda: defaultdict(float))
    for r in part:
        c[r["Queue_Id"]][cat(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for q, d in sorted(c.items()):
        print(f"  {name} queue {q}:", {k: round(v) for k, v in sorted(d.items(), key=lambda kv: -kv[1])})
