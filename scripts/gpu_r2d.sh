#!/bin/bash
# Round-2 pass D: numerics of the changed kernels (head backward with fused BN partials,
# 96-channel resident-weight variant), then the bench and a serial kernel trace.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_gpu.py tests/test_data_gpu.py \
  tests/test_properties.py -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pytest_d.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/pytest_d.log | head -20; tail -2 gpurun_out/pytest_d.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes dgrad --only dec1 > gpurun_out/micro_d.txt 2>&1 || { tail -20 gpurun_out/micro_d.txt; exit 2; }
cat gpurun_out/micro_d.txt
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 3; }
cat gpurun_out/bench.json
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --steps 5 --warmup 3 --schedule serial > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 5; }
f=$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)
python scripts/trace_summary.py "$f" 7 > gpurun_out/prof_summary.txt 2>&1
python scripts/stream_summary.py "$f" >> gpurun_out/prof_summary.txt 2>&1
cat gpurun_out/prof_summary.txt
exit $rc
