#!/bin/bash
# round 2, pass J: host run-ahead bound (DDLPC_MAX_INFLIGHT) vs unbounded, fresh processes
# alternated; 1024^2 x 128 overlap with a tighter side-stream lag budget
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2j
mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2 3; do
  run bounded_$i 200 python -u bench.py
  run unbounded_$i 200 env DDLPC_MAX_INFLIGHT=0 python -u bench.py
done
run t1024_b128_lag16 400 env DDLPC_SIDE_LAG_GB=16 python -u bench.py --tile 1024 --batch 128 --steps 3 --warmup 3 --schedule overlap --heartbeat 30
