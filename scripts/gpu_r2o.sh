#!/bin/bash
# round 2, pass O: 8-wave 256x128 conv tiles (cfg 4, one workgroup per CU) vs 4-wave 128x128
# tiles (cfg 2, two workgroups per CU: barriers of one overlap the other's compute)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2o
mkdir -p $O
export TMPDIR=/tmp
for v in 1 0; do
  DDLPC_CONV_CFG4=$v timeout -k 10 150 python -u scripts/conv_micro.py --batch 128 --passes fwd,dgrad > $O/cfg4_$v.txt 2>&1 || exit 1
done
paste <(grep -v amdgpu $O/cfg4_1.txt | cut -c1-40) <(grep -v amdgpu $O/cfg4_0.txt | cut -c16-40)
