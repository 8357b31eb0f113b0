#!/bin/bash
# round 2 session 2, pass K: occupancy knobs of the two-stream schedule (same box, A B A B)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2k
mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
run base 200 python -u bench.py
run wpc1 200 env DDLPC_WGRAD_WG_PER_CU=1 python -u bench.py
run wpc3 200 env DDLPC_WGRAD_WG_PER_CU=3 python -u bench.py
run base2 200 python -u bench.py
run wpc1b 200 env DDLPC_WGRAD_WG_PER_CU=1 python -u bench.py
run wpc4 200 env DDLPC_WGRAD_WG_PER_CU=4 python -u bench.py
run prio 200 env DDLPC_SIDE_PRIORITY=0 python -u bench.py
run base3 200 python -u bench.py
