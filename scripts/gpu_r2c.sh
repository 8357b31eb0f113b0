#!/bin/bash
# Round-2 pass C: re-check the fixed tests, BN-backward and conv fwd/dgrad per-layer rates
# at batch 128, and a serial-schedule kernel trace of the bench step.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_data_gpu.py tests/test_unet_gpu.py -m gpu -v \
  --timeout 150 --timeout-method thread > gpurun_out/pytest_c.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_c.log | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 200 python -u scripts/bn_micro.py > gpurun_out/bn_micro.txt 2>&1 || { tail -20 gpurun_out/bn_micro.txt; exit 2; }
cat gpurun_out/bn_micro.txt
rm -rf gpurun_out/prof_bn
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bn -o bn -- \
  python3 scripts/bn_micro.py --iters 3 > gpurun_out/prof_bn.log 2>&1 || { tail -20 gpurun_out/prof_bn.log; exit 3; }
f=$(find gpurun_out/prof_bn -name '*kernel_stats.csv' | head -1); head -12 "$f"
timeout -k 10 300 python -u scripts/conv_micro.py --batch 128 --passes fwd,dgrad > gpurun_out/micro_fd.txt 2>&1 || { tail -20 gpurun_out/micro_fd.txt; exit 4; }
cat gpurun_out/micro_fd.txt
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --steps 5 --warmup 3 --schedule serial > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 5; }
grep '^{' gpurun_out/prof.log | cut -c1-200
f=$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)
python scripts/trace_summary.py "$f" 7 > gpurun_out/prof_summary.txt 2>&1
python scripts/stream_summary.py "$f" >> gpurun_out/prof_summary.txt 2>&1
cat gpurun_out/prof_summary.txt
exit $rc
