#!/bin/bash
# GPU validation: kernel numerics, end-to-end engine parity, and a short bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
python scripts/build_ext.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_unet_gpu.py -q -m gpu -rA > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --impl hip --batch 32 --steps 10 --warmup 3 > gpurun_out/bench_hip.json 2> gpurun_out/bench_hip.err || { tail -20 gpurun_out/bench_hip.err; exit 3; }
cat gpurun_out/bench_hip.json
if [ -n "$PROF" ]; then
  bash scripts/gpu_prof.sh > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 4; }
  python scripts/trace_summary.py gpurun_out/prof/run_kernel_trace.csv 7 > gpurun_out/prof_summary.txt && cat gpurun_out/prof_summary.txt
fi
