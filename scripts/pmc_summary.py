#!/usr/bin/env python
"""Per-dispatch PMC summary of a rocprofv3 --pmc counter_collection.csv (conv micro runs)."""
import csv
import sys
from collections import OrderedDict, defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
RAW = "--raw" in sys.argv
agg = OrderedDict()
for r in rows:
    k = (int(r["Dispatch_Id"]), r["Kernel_Name"].replace("void ", "").replace("ddlpc::(anonymous namespace)::", "").split("(")[0][:44])
    agg.setdefault(k, defaultdict(float))[r["Counter_Name"]] += float(r["Counter_Value"])
for (d, name), c in agg.items():
    if "conv" not in name and "wgrad" not in name and "head" not in name:
        continue
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    parts = [f"{d:5d} {name:44s}"]
    if RAW:
        print(" ".join(parts + [f"{k}={v:.4g}" for k, v in sorted(c.items())]))
        continue
    if "GRBM_GUI_ACTIVE" in c and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        # MFMA busy per SIMD-cycle (256 CUs x 4 SIMDs)
        parts.append(f"mfma_util={c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['GRBM_GUI_ACTIVE'] * 1024):.3f}")
    for key in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS"):
        if key in c:
            parts.append(f"{key[3:]}={c[key] / wc:.2f}")
    for key in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT",
                "SQ_INSTS_SALU", "SQ_BUSY_CYCLES"):
        if key in c:
            parts.append(f"{key[3:]}={c[key]:.3g}")
    print(" ".join(parts))
