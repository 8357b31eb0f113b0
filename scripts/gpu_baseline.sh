#!/bin/bash
# In-house baseline: stock PyTorch-ROCm (MIOpen) U-Net, bf16 autocast, channels_last.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 32 64; do
  timeout -k 10 400 python bench.py --impl torch --batch $B --steps 10 --warmup 5 > gpurun_out/base_b$B.json 2> gpurun_out/base_b$B.err || exit $?
  cat gpurun_out/base_b$B.json
done
