#!/bin/bash
# round 2 session 2, pass M: head kernels' occupancy (workgroups per CU of the persistent
# fused forward/statistics kernel): serial traces per setting + bench
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2m
mkdir -p $O
export TMPDIR=/tmp
for pc in 0 4 8; do
  timeout -k 10 300 env DDLPC_HEAD_BWD_PER_CU=$pc rocprofv3 --kernel-trace --output-format csv -d $O/prof$pc -o run -- \
    python3 bench.py --steps 5 --warmup 3 --schedule serial > $O/prof$pc.log 2>&1 || { tail -20 $O/prof$pc.log; exit 4; }
  f=$(find $O/prof$pc -name '*kernel_trace.csv' | head -1)
  echo "== per_cu=$pc"; python scripts/trace_summary.py "$f" 7 v | grep -E "head_" | head -3
done
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
run b0 200 python -u bench.py
run b4 200 env DDLPC_HEAD_BWD_PER_CU=4 python -u bench.py
run b0b 200 python -u bench.py
run b4b 200 env DDLPC_HEAD_BWD_PER_CU=4 python -u bench.py
