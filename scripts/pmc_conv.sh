#!/bin/bash
# SQ counters of the 3x3 conv kernels on one layer (conv_micro), one rocprofv3 --pmc pass:
#   scripts/pmc_conv.sh OUTDIR LAYER [conv_micro args...]
#   PMC="..." overrides the counter set (one pass: <= 8 SQ_ counters + GRBM_GUI_ACTIVE);
#   PMC=mix: the instruction mix (VALU / SALU / LDS / MFMA / VMEM / SMEM / branch)
set -eo pipefail
out=$1; layer=$2; shift 2
mkdir -p "$out"
export TMPDIR=/tmp
case "${PMC:-}" in
  "") ctr="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" ;;
  mix) ctr="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES GRBM_GUI_ACTIVE" ;;
  *) ctr="$PMC" ;;
esac
timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$out/pmc" -o run -- \
  python3 scripts/conv_micro.py --batch 128 --iters 3 --only "$layer" "$@" > "$out/micro.log" 2>&1
f=$(find "$out/pmc" -name '*counter_collection.csv' | head -1)
python scripts/pmc_summary.py "$f" --raw > "$out/summary.txt"
python scripts/pmc_summary.py "$f" >> "$out/summary.txt"
cat "$out/summary.txt"
