#!/bin/bash
# round 2, pass S: v3 weight gradient pixel tile for the concat layers (96 vs 128 vs v2),
# then the MIOpen 3-D baseline (config #5)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 150 python -u scripts/conv_micro.py --batch 128 --passes wgrad --only .a > $O/w128.txt 2>&1 || exit 1
DDLPC_WGRAD3_PT64=96 timeout -k 10 150 python -u scripts/conv_micro.py --batch 128 --passes wgrad --only .a > $O/w96.txt 2>&1 || exit 1
paste <(grep -v amdgpu $O/w128.txt | cut -c1-40) <(grep -v amdgpu $O/w96.txt | cut -c16-40)
CFG=torch_d3 bash scripts/gpu_cfg_r2.sh
