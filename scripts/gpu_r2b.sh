#!/bin/bash
# Round-2 pass B: full GPU suite (no -x: see every failure), per-layer wgrad timings +
# LDS-conflict counters of the re-laid-out weight-gradient kernel, then the driver bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | grep -v PASSED | head -30
tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u scripts/conv_micro.py --batch 128 --passes wgrad > gpurun_out/micro_wgrad.txt 2>&1 || { tail -20 gpurun_out/micro_wgrad.txt; exit 2; }
cat gpurun_out/micro_wgrad.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc_wg -o pmc -- python3 scripts/conv_micro.py --batch 128 --iters 2 --passes wgrad > gpurun_out/pmc_wg.log 2>&1 || { tail -20 gpurun_out/pmc_wg.log; exit 3; }
f=$(find gpurun_out/pmc_wg -name "*counter_collection.csv" | sort | tail -n 1)
python scripts/pmc_summary.py "$f" > gpurun_out/pmc_wg_summary.txt 2>&1; head -30 gpurun_out/pmc_wg_summary.txt
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 4; }
cat gpurun_out/bench.json
exit $rc
