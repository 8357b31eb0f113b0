#!/usr/bin/env python
"""Per-step GPU occupancy of a rocprofv3 kernel trace (results .db or kernel_trace.csv).

For every training step (between consecutive Adam launches): wall time, time with at least
one kernel running (union over queues), and the idle gaps longer than --min-gap-us with the
kernels on either side — where a step loses time that no kernel accounts for.

    python scripts/step_gaps.py gpurun_out/prof/run_results.db [--min-gap-us 20]
"""
import argparse
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def load(path):
    if path.endswith(".db"):
        import sqlite3
        c = sqlite3.connect(path)
        return [(n, int(s), int(e), str(q)) for n, s, e, q in
                c.execute("select name, start, end, queue_id from kernels order by start")]
    return sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"])
                   for r in csv.DictReader(open(path))), key=lambda t: t[1])


def short(n):
    n = n.replace("void ", "").replace("ddlpc::(anonymous namespace)::", "")
    return n.split("(")[0][:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--min-gap-us", type=float, default=20.0)
    a = ap.parse_args()
    rows = load(a.trace)
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r[0]]
    for si in range(1, len(adam)):
        seg = rows[adam[si - 1] + 1: adam[si] + 1]
        # the step starts where the previous Adam ended (host gaps between steps count)
        t0, t1 = rows[adam[si - 1]][2], max(r[2] for r in seg)
        busy, cur_s, cur_e = 0, None, None
        gaps = []
        last = rows[adam[si - 1]][0]
        if seg[0][1] - t0 >= a.min_gap_us * 1e3:
            gaps.append(((seg[0][1] - t0) / 1e3, short(last), short(seg[0][0])))
        for n, s, e, q in seg:
            if cur_e is None:
                cur_s, cur_e, last = s, e, n
                continue
            if s > cur_e:
                busy += cur_e - cur_s
                if (s - cur_e) / 1e3 >= a.min_gap_us:
                    gaps.append(((s - cur_e) / 1e3, short(last), short(n)))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
            if e >= cur_e:
                last = n
        busy += cur_e - cur_s
        print(f"step {si}: wall {(t1 - t0) / 1e6:.3f} ms, some kernel running {busy / 1e6:.3f} ms, "
              f"idle {(t1 - t0 - busy) / 1e6:.3f} ms, kernels {len(seg)}")
        for g, p, nx in sorted(gaps, reverse=True)[:8]:
            print(f"    gap {g:8.1f} us  after {p:48s} before {nx}")


if __name__ == "__main__":
    main()
