#!/bin/bash
# SQ counters of the fused head kernels (head_micro), one rocprofv3 --pmc pass:
#   scripts/pmc_head.sh OUTDIR [head_micro args...]   (PMC="..." overrides the counter set)
set -eo pipefail
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
ctr="${PMC:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE}"
timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$out/pmc" -o run -- \
  python3 scripts/head_micro.py --iters 3 "$@" > "$out/micro.log" 2>&1
f=$(find "$out/pmc" -name '*counter_collection.csv' | head -1)
python scripts/pmc_summary.py "$f" --raw > "$out/summary.txt"
python scripts/pmc_summary.py "$f" >> "$out/summary.txt"
cat "$out/summary.txt"
