#!/bin/bash
# round 2 session 2, pass Y: re-check the scheduling / tiling knobs against the current
# kernel mix (bench at the default config, default bracketing the variants)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2y
mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json | cut -c1-70; [ $rc -eq 0 ] || exit $rc; }
run def_a 200 python -u bench.py
run sideprio0 200 env DDLPC_SIDE_PRIORITY=0 python -u bench.py
run sideconvt0 200 env DDLPC_SIDE_CONVT=0 python -u bench.py
run wgpc1 200 env DDLPC_WGRAD_WG_PER_CU=1 python -u bench.py
run wgpc3 200 env DDLPC_WGRAD_WG_PER_CU=3 python -u bench.py
run inflight3 200 env DDLPC_MAX_INFLIGHT=3 python -u bench.py
run resdepth2 200 env DDLPC_RES_DEPTH=2 python -u bench.py
run def_b 200 python -u bench.py
