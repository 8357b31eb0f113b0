#!/usr/bin/env python
"""Per-kernel register / scratch / occupancy table of a csrc/*.hip unit (gfx950).

    python scripts/kernel_resources.py csrc/head_ce.hip [name-filter]

Compiles the unit with ``-Rpass-analysis=kernel-resource-usage`` (no GPU needed) and
prints one line per kernel: VGPRs, AGPRs, SGPRs, scratch bytes per lane, LDS bytes and
waves per SIMD.  Any scratch use on a hot kernel is a spill to fix before measuring.
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = os.path.abspath(sys.argv[1])
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I",
           os.path.join(ROOT, "csrc"), "-c", src, "-o", "/dev/null",
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp").stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (?:\s*)(.+?): (.+?) \[-Rpass", line)
        if not m:
            continue
        key, val = m.group(1).strip(), m.group(2).strip()
        if key == "Function Name":
            cur = {"name": val}
            rows.append(cur)
        elif cur is not None:
            cur[key] = val
    for r in rows:
        name = r["name"]
        if filt and filt not in name:
            continue
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        dem = re.sub(r"ddlpc::\(anonymous namespace\)::", "", dem)
        dem = re.sub(r"\(.*\)$", "", dem)
        print(f"{dem[:72]:72s} v{r.get('VGPRs', '?'):>4} a{r.get('AGPRs', '?'):>4} "
              f"s{r.get('TotalSGPRs', '?'):>4} scratch{r.get('ScratchSize [bytes/lane]', '?'):>5} "
              f"lds{r.get('LDS Size [bytes/block]', '?'):>6} occ{r.get('Occupancy [waves/SIMD]', '?'):>2}")


if __name__ == "__main__":
    main()
