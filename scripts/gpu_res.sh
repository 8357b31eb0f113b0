#!/bin/bash
# resident-weight conv kernel: numerics + per-layer timing (res on / off)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
python scripts/build_ext.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "conv3" > gpurun_out/pytest_res.log 2>&1 || { tail -40 gpurun_out/pytest_res.log; exit 2; }
tail -3 gpurun_out/pytest_res.log
timeout -k 10 300 python scripts/conv_micro.py --passes fwd,dgrad $MICRO_ARGS > gpurun_out/micro_res.txt 2>&1 || { tail -20 gpurun_out/micro_res.txt; exit 3; }
DDLPC_CONV_RES=0 timeout -k 10 300 python scripts/conv_micro.py --passes fwd,dgrad $MICRO_ARGS > gpurun_out/micro_nores.txt 2>&1 || { tail -20 gpurun_out/micro_nores.txt; exit 4; }
paste gpurun_out/micro_res.txt gpurun_out/micro_nores.txt | grep -v amdgpu.ids
