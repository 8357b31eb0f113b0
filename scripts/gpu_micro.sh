#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
python scripts/build_ext.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 300 python scripts/conv_micro.py $MICRO_ARGS > gpurun_out/micro.txt 2>&1 || { tail -20 gpurun_out/micro.txt; exit 2; }
cat gpurun_out/micro.txt
if [ -n "$PMC" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc ${PMC_CTRS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT} --output-format csv -d gpurun_out/pmc -o pmc -- python3 scripts/conv_micro.py --iters 2 $MICRO_ARGS > gpurun_out/pmc.log 2>&1 || { tail -20 gpurun_out/pmc.log; exit 3; }
  ls gpurun_out/pmc
fi
