#!/bin/bash
# round 2, pass N (diagnostic): streaming-conv time with the weight / halo DMA skipped
# (wrong results, timing only) -> what the operand streams cost
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2n
mkdir -p $O
export TMPDIR=/tmp
for d in 0 1 2 3; do
  DDLPC_DIAG_CONV=$d timeout -k 10 150 python -u scripts/conv_micro.py --batch 128 --passes fwd,dgrad > $O/diag$d.txt 2>&1 || exit 1
  echo "== diag=$d"; grep -v amdgpu $O/diag$d.txt | grep -E "enc3.b|enc4.b|dec4.a|dec3.a|totals"
done
