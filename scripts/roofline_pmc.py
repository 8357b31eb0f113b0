#!/usr/bin/env python
"""Per-kernel HBM traffic and achieved bandwidth of the last training step, from two
rocprofv3 --pmc passes over the same bench command (FETCH_SIZE and WRITE_SIZE, kilobytes,
each in its own run).  Step = dispatches between the last two Adam launches of each run.

usage: roofline_pmc.py fetch_counter_collection.csv write_counter_collection.csv"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "").replace("ddlpc::", "")
    return re.sub(r"\(.*$", "", n)[:64]


def last_step(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    seg = rows[idx[-2] + 1:idx[-1] + 1] if len(idx) >= 2 else rows
    agg = defaultdict(lambda: [0, 0.0, 0.0])          # launches, KB, us
    for r in seg:
        a = agg[short(r["Kernel_Name"])]
        a[0] += 1
        a[1] += float(r["Counter_Value"])
        a[2] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return agg


f = last_step(sys.argv[1], "FETCH_SIZE")
w = last_step(sys.argv[2], "WRITE_SIZE")
tot_t = tot_b = 0.0
print(f"{'us/step':>8} {'n':>3} {'read GB':>8} {'write GB':>8} {'TB/s':>6}  kernel")
for k in sorted(f, key=lambda k: -f[k][2]):
    n, rkb, t = f[k]
    wkb = w.get(k, [0, 0.0, 0.0])[1]
    gb_r, gb_w = rkb / 1e6, wkb / 1e6
    tot_t += t
    tot_b += gb_r + gb_w
    if t >= 20:
        print(f"{t:8.1f} {n:3d} {gb_r:8.3f} {gb_w:8.3f} {(gb_r + gb_w) / (t * 1e-6) / 1e3:6.2f}  {k}")
print(f"step: {tot_t / 1e3:.2f} ms of kernels (serialised by the counter run), "
      f"{tot_b:.1f} GB of HBM traffic, {tot_b / (tot_t * 1e-6) / 1e3:.2f} TB/s average")
