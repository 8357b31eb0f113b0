#!/bin/bash
# rocprofv3 kernel trace + stats of a short HIP-path bench (summary copied to profiles/).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
B=${B:-32}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 bench.py --impl ${IMPL:-hip} --batch $B --steps 5 --warmup 2 > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err || { tail -20 gpurun_out/prof_bench.err; exit 1; }
cat gpurun_out/prof_bench.json
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
echo "stats: $f"
head -40 "$f"
