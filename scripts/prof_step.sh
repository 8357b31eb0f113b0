#!/bin/bash
# rocprofv3 kernel trace of a batch-128 serial-schedule bench step + per-kernel summary:
#   scripts/prof_step.sh OUTDIR [bench args...]   (knobs via DDLPC_* environment)
set -eo pipefail
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 bench.py --steps 5 --warmup 3 --schedule serial "$@" > "$out/bench.log" 2>&1
f=$(find "$out/trace" -name '*kernel_trace.csv' | head -1)
python scripts/trace_summary.py "$f" 5 > "$out/summary.txt" 2>&1
head -3 "$out/summary.txt"
