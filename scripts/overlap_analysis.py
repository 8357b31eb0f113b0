#!/usr/bin/env python
"""How much of the weight-gradient side stream actually overlaps the compute stream.

Reads a rocprofv3 kernel_trace.csv of an overlapped-schedule run and, for the last training
step (between the last two Adam launches), reports per queue: busy time, the wall time in
which both queues have a kernel running, and per side-stream kernel name how much of its
time ran concurrently with a main-stream kernel (the rest serialised the step).
Usage: overlap_analysis.py kernel_trace.csv [top]
"""
import csv
import sys
from collections import defaultdict


def intervals(rows):
    return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)


def union(iv):
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], e))
        else:
            out.append((s, e))
    return out


def overlap(s, e, merged):
    t = 0
    for a, b in merged:
        if b <= s:
            continue
        if a >= e:
            break
        t += min(b, e) - max(a, s)
    return t


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    lo, hi = (idx[-2] + 1, idx[-1] + 1) if len(idx) >= 2 else (0, len(rows))
    seg = rows[lo:hi]
    queues = defaultdict(list)
    for r in seg:
        queues[r["Queue_Id"]].append(r)
    # the compute stream launches the Adam kernel
    main_q = rows[idx[-1]]["Queue_Id"] if idx else max(queues, key=lambda q: len(queues[q]))
    t0 = min(int(r["Start_Timestamp"]) for r in seg)
    t1 = max(int(r["End_Timestamp"]) for r in seg)
    mm = union(intervals(queues[main_q]))
    print(f"step wall {(t1 - t0) / 1e3:.1f} us, main queue {main_q} busy "
          f"{sum(b - a for a, b in mm) / 1e3:.1f} us")
    allu = union(intervals(seg))
    print(f"any-kernel busy {sum(b - a for a, b in allu) / 1e3:.1f} us "
          f"(idle {((t1 - t0) - sum(b - a for a, b in allu)) / 1e3:.1f} us)")
    for q, rs in queues.items():
        if q == main_q:
            continue
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs)
        ov = sum(overlap(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), mm) for r in rs)
        print(f"queue {q}: busy {busy / 1e3:.1f} us, concurrent with main {ov / 1e3:.1f} us "
              f"({100.0 * ov / max(busy, 1):.0f}%), serialised {(busy - ov) / 1e3:.1f} us")
        per = defaultdict(lambda: [0, 0, 0])
        for r in rs:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            n = r["Kernel_Name"].replace("void ", "").replace("ddlpc::(anonymous namespace)::", "")
            n = n.split("(")[0][:48]
            per[n][0] += e - s
            per[n][1] += overlap(s, e, mm)
            per[n][2] += 1
        for n, (b, o, c) in sorted(per.items(), key=lambda kv: -kv[1][0])[:top]:
            print(f"   {b / 1e3:8.1f} us  concurrent {o / 1e3:8.1f}  x{c:<3d} {n}")


if __name__ == "__main__":
    main()
