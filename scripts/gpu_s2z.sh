#!/bin/bash
# round 2 session 2, pass Z: per-kernel HBM bytes of one training step (FETCH_SIZE and
# WRITE_SIZE in separate counter runs) -> achieved bandwidth per kernel class
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2z
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 2 --warmup 2 --schedule serial > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; exit 3; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- python3 bench.py --steps 2 --warmup 2 --schedule serial > $O/write.log 2>&1 || { tail -20 $O/write.log; exit 4; }
ff=$(find $O/fetch -name '*counter_collection.csv' | head -1)
fw=$(find $O/write -name '*counter_collection.csv' | head -1)
python scripts/roofline_pmc.py "$ff" "$fw" > $O/roofline.txt 2>&1; cat $O/roofline.txt
rm -f "$ff" "$fw"
