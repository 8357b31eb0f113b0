#!/bin/bash
# numerics (pytest -k $TESTS) + per-layer conv micro-benchmark A/B: default vs $AB_ENV
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
python scripts/build_ext.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "${TESTS:-conv3}" > gpurun_out/pytest_ab.log 2>&1 || { tail -40 gpurun_out/pytest_ab.log; exit 2; }
tail -2 gpurun_out/pytest_ab.log
timeout -k 10 300 python scripts/conv_micro.py --passes ${PASSES:-fwd,dgrad,wgrad} $MICRO_ARGS > gpurun_out/micro_a.txt 2>&1 || { tail -20 gpurun_out/micro_a.txt; exit 3; }
if [ -n "$AB_ENV" ]; then
  env $AB_ENV timeout -k 10 300 python scripts/conv_micro.py --passes ${PASSES:-fwd,dgrad,wgrad} $MICRO_ARGS > gpurun_out/micro_b.txt 2>&1 || { tail -20 gpurun_out/micro_b.txt; exit 4; }
  paste gpurun_out/micro_a.txt gpurun_out/micro_b.txt | grep -v amdgpu.ids
else
  grep -v amdgpu.ids gpurun_out/micro_a.txt
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python bench.py --batch 32 --steps 10 --warmup 3 > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { tail -20 gpurun_out/bench_ab.err; exit 5; }
  cat gpurun_out/bench_ab.json
fi
