#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
python scripts/build_ext.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_unet_gpu.py tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 2; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --batch 32 --steps 20 --warmup 5 > gpurun_out/bench_eager.json 2> gpurun_out/bench_eager.err || { tail -20 gpurun_out/bench_eager.err; exit 3; }
cat gpurun_out/bench_eager.json
timeout -k 10 300 python bench.py --batch 32 --steps 20 --warmup 5 --hip-graph 1 > gpurun_out/bench_graph.json 2> gpurun_out/bench_graph.err || { tail -20 gpurun_out/bench_graph.err; exit 4; }
cat gpurun_out/bench_graph.json
