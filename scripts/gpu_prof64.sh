#!/bin/bash
# rocprofv3 kernel trace of the default bench config + per-stream/category summary
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
python scripts/build_ext.py > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --steps 5 --warmup 3 $BENCH_ARGS > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 2; }
grep '^{' gpurun_out/prof.log
f=$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)
python scripts/trace_summary.py "$f" 7 > gpurun_out/prof_summary.txt 2>&1
python scripts/stream_summary.py "$f" >> gpurun_out/prof_summary.txt 2>&1
cat gpurun_out/prof_summary.txt
