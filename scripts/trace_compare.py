#!/usr/bin/env python
"""Per-kernel time of the last training step of two rocprofv3 traces, normalised per image.

    python scripts/trace_compare.py A.db 32 B.db 64

prints, per kernel name (template arguments kept), µs per image in A and B and the ratio —
which kernels make a larger batch slower per image.
"""
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from step_gaps import load, short  # noqa: E402


def last_step(path):
    rows = load(path)
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r[0]]
    seg = rows[adam[-2] + 1: adam[-1] + 1] if len(adam) >= 2 else rows
    agg = defaultdict(float)
    for n, s, e, _q in seg:
        agg[short(n)] += (e - s) / 1e3
    wall = (seg[-1][2] - rows[adam[-2]][2]) / 1e3 if len(adam) >= 2 else 0.0
    return agg, wall


def main():
    a_path, a_n, b_path, b_n = sys.argv[1], float(sys.argv[2]), sys.argv[3], float(sys.argv[4])
    A, wa = last_step(a_path)
    B, wb = last_step(b_path)
    print(f"step wall: A {wa / 1e3:.2f} ms ({wa / a_n:.1f} us/img), B {wb / 1e3:.2f} ms ({wb / b_n:.1f} us/img)")
    rows = []
    for k in set(A) | set(B):
        pa, pb = A.get(k, 0.0) / a_n, B.get(k, 0.0) / b_n
        rows.append((pb - pa, k, pa, pb))
    print(f"{'kernel':48s} {'A us/img':>9s} {'B us/img':>9s} {'B-A':>8s}")
    for d, k, pa, pb in sorted(rows, reverse=True)[:20]:
        print(f"{k:48s} {pa:9.2f} {pb:9.2f} {d:8.2f}")
    print(f"{'total':48s} {sum(A.values()) / a_n:9.2f} {sum(B.values()) / b_n:9.2f}")


if __name__ == "__main__":
    main()
