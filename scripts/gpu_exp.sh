#!/bin/bash
# conv forward experiments: debug knobs (1 = no weight traffic, 2 = no halo traffic,
# 4 = no MFMA, 8 = no stage barrier) and persistence / split-K overrides
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
python scripts/build_ext.py > gpurun_out/build.log 2>&1 || exit 1
for cfg in ${DBGS:-0 16 32 48 52 60}; do
  echo "== DBG=$cfg"
  DDLPC_CONV_DBG=$cfg timeout -k 10 120 python scripts/conv_micro.py --passes fwd --only "$ONLY" || exit 2
done
for pb in ${PBS:-}; do
  echo "== PERSIST=$pb"
  DDLPC_CONV_PERSIST=$pb timeout -k 10 120 python scripts/conv_micro.py --passes fwd --only "$ONLY" || exit 2
done
if [ -n "$LAT" ] && [ -x tools/dma_latency ]; then timeout -k 10 60 ./tools/dma_latency || exit 3; fi
