#!/bin/bash
# weight-gradient kernels: per-layer timing at batch 128 + two PMC passes (SQ, TCC)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
python scripts/build_ext.py > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 200 python scripts/conv_micro.py --batch 128 --passes ${PASSES:-wgrad} --iters 10 > gpurun_out/wg_time.log 2>&1 || { tail -20 gpurun_out/wg_time.log; exit 2; }
cat gpurun_out/wg_time.log
rm -rf gpurun_out/pmc1 gpurun_out/pmc2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc1 -o run -- python3 scripts/conv_micro.py --batch 128 --passes ${PASSES:-wgrad} --iters 1 --only ${ONLY:-b} > gpurun_out/pmc1.log 2>&1 || { tail -20 gpurun_out/pmc1.log; exit 3; }
f=$(find gpurun_out/pmc1 -name '*counter_collection.csv' | head -1)
python scripts/pmc_summary.py "$f" > gpurun_out/pmc1_summary.txt; cat gpurun_out/pmc1_summary.txt
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc2 -o run -- python3 scripts/conv_micro.py --batch 128 --passes ${PASSES:-wgrad} --iters 1 --only ${ONLY:-b} > gpurun_out/pmc2.log 2>&1 || { tail -20 gpurun_out/pmc2.log; exit 4; }
f=$(find gpurun_out/pmc2 -name '*counter_collection.csv' | head -1)
python - "$f" <<'PY'
import csv, sys, collections
agg = collections.OrderedDict()
for r in csv.DictReader(open(sys.argv[1])):
    k = (int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ddlpc::(anonymous namespace)::", "")[:40])
    agg.setdefault(k, collections.defaultdict(float))[r["Counter_Name"]] += float(r["Counter_Value"])
for (d, n), c in agg.items():
    h, m = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
    print(f"{d:5d} {n:40s} hit={h:.3g} miss={m:.3g} hitrate={h / max(h + m, 1):.2f} missMB={m * 128 / 1e6:.1f}")
PY
