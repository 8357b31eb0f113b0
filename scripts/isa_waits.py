#!/usr/bin/env python
"""Histogram of the LDS waits in front of the MFMAs of each kernel in a gfx950 assembly file.

    hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S csrc/X.hip -o /tmp/X.s
    python scripts/isa_waits.py /tmp/X.s [kernel-name-filter]

For every v_mfma the nearest preceding `s_waitcnt` (within the same basic block) is classified
(and, per kernel, the VALU / SALU instructions inside basic blocks that hold MFMAs are counted:
their ratio to the MFMAs flags per-fragment address arithmetic in the inner loops):
`lgkmcnt(0)` in front of an MFMA means no LDS read is in flight across it — the fragment
pipeline is one deep and the read latency is exposed; `vmcnt(0)` in a compute loop drains the
LDS-DMA ring.  Prints, per kernel: MFMAs, waits by kind, and the share behind lgkmcnt(0).
"""
import re
import sys
from collections import Counter


def main():
    lines = open(sys.argv[1]).read().split("\n")
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    kern, stats = None, {}
    last_wait = None
    blk = Counter()                                  # the current basic block's mix

    def close_block():
        if kern is not None and blk["mfma"]:
            stats[kern]["loop_valu"] += blk["valu"]
            stats[kern]["loop_salu"] += blk["salu"]
        blk.clear()

    for ln in lines:
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            close_block()
            kern = m.group(1)
            stats.setdefault(kern, Counter())
            last_wait = None
            continue
        if kern is None:
            continue
        t = ln.strip()
        if t.startswith("v_mfma"):
            blk["mfma"] += 1
        elif t.startswith("v_"):
            blk["valu"] += 1
        elif t.startswith("s_") and not t.startswith(("s_waitcnt", "s_nop", "s_setprio", "s_barrier", "s_cbranch", "s_branch")):
            blk["salu"] += 1
        if t.startswith(".LBB") or t.startswith("s_cbranch") or t.startswith("s_branch"):
            close_block()
            last_wait = None
        elif t.startswith("s_waitcnt"):
            last_wait = t
        elif t.startswith("v_mfma"):
            c = stats[kern]
            c["mfma"] += 1
            if last_wait is None:
                c["no_wait"] += 1
            else:
                lg = re.search(r"lgkmcnt\((\d+)\)", last_wait)
                vm = re.search(r"vmcnt\((\d+)\)", last_wait)
                if lg:
                    c["lgkm0" if lg.group(1) == "0" else "lgkmN"] += 1
                if vm and vm.group(1) == "0":
                    c["vm0"] += 1
            last_wait = None
    for k, c in stats.items():
        if not c["mfma"] or filt not in k:
            continue
        name = re.sub(r"^_ZN5ddlpc12_GLOBAL__N_1\d+", "", k)[:70]
        print(f"{name:70s} mfma {c['mfma']:5d}  lgkm(0) {c['lgkm0']:4d} ({c['lgkm0'] / c['mfma']:.0%})"
              f"  lgkm(N) {c['lgkmN']:4d}  vm(0) {c['vm0']:3d}  none {c['no_wait']:4d}"
              f"  loop VALU/MFMA {c['loop_valu'] / c['mfma']:.2f}  SALU/MFMA {c['loop_salu'] / c['mfma']:.2f}")


if __name__ == "__main__":
    main()
