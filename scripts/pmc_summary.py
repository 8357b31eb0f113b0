#!/usr/bin/env python
"""Per-dispatch PMC summary of a rocprofv3 --pmc counter_collection.csv (conv micro runs).

Normalisation (MI355X_MICROARCH.md, 'PMC units'): rocprofv3 reports GRBM_GUI_ACTIVE summed
over the 8 XCDs, so the kernel's cycle count is GRBM_GUI_ACTIVE / 8 and the effective clock
is that over the dispatch's wall time; SQ_VALU_MFMA_BUSY_CYCLES counts MFMA cycles summed
over all SIMDs (32 per v_mfma_f32_32x32x16_bf16, 16 per 16x16x32), so the MFMA utilisation
is MFMA_BUSY / (cycles x 256 CUs x 4 SIMDs).  (Round 3 divided by the XCD-summed
GRBM_GUI_ACTIVE, which understated the utilisation 8x.)  SQ_WAIT_* / SQ_ACTIVE_INST_* are
per-wave ratios against SQ_WAVE_CYCLES (same units)."""
import csv
import sys
from collections import OrderedDict, defaultdict

N_XCD, N_CU, SIMD_PER_CU = 8, 256, 4

rows = list(csv.DictReader(open(sys.argv[1])))
RAW = "--raw" in sys.argv
agg = OrderedDict()
span = {}
for r in rows:
    k = (int(r["Dispatch_Id"]), r["Kernel_Name"].replace("void ", "").replace("ddlpc::(anonymous namespace)::", "").split("(")[0][:44])
    agg.setdefault(k, defaultdict(float))[r["Counter_Name"]] += float(r["Counter_Value"])
    span[k] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for key, c in agg.items():
    d, name = key
    if "conv" not in name and "wgrad" not in name and "head" not in name and "bn_" not in name:
        continue
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    parts = [f"{d:5d} {name:44s}"]
    if RAW:
        print(" ".join(parts + [f"{k}={v:.4g}" for k, v in sorted(c.items())]))
        continue
    ns = span.get(key, 0)
    parts.append(f"us={ns / 1e3:.1f}")
    if "GRBM_GUI_ACTIVE" in c:
        cyc = c["GRBM_GUI_ACTIVE"] / N_XCD
        if ns > 0:
            parts.append(f"clk_ghz={cyc / ns:.2f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            parts.append(f"mfma_util={c['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * N_CU * SIMD_PER_CU):.3f}")
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
              "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS"):
        if k in c:
            parts.append(f"{k[3:]}={c[k] / wc:.2f}")
    for k in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT",
              "SQ_INSTS_SALU", "SQ_BUSY_CYCLES"):
        if k in c:
            parts.append(f"{k[3:]}={c[k]:.3g}")
    print(" ".join(parts))
