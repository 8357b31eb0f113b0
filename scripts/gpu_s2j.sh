#!/bin/bash
# round 2 session 2, pass J: deferred encoder skip at the 256^2 level only (A/B), engine
# numerics with it, and 1024^2 x 128 with the retry-aware schedule probe
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2j
mkdir -p $O
export TMPDIR=/tmp
DDLPC_DEFER_SKIP=1 DDLPC_DEFER_SKIP_LEVELS=0 timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_unet_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run bench_a 200 python -u bench.py
run bench_s0 200 env DDLPC_DEFER_SKIP=1 DDLPC_DEFER_SKIP_LEVELS=0 python -u bench.py
run bench_b 200 python -u bench.py
run bench_s0b 200 env DDLPC_DEFER_SKIP=1 DDLPC_DEFER_SKIP_LEVELS=0 python -u bench.py
run bench_s01 200 env DDLPC_DEFER_SKIP=1 DDLPC_DEFER_SKIP_LEVELS=0,1 python -u bench.py
run t1024_b128 400 python -u bench.py --tile 1024 --batch 128 --steps 3 --warmup 3
run t1024_b64 300 python -u bench.py --tile 1024 --batch 64 --steps 4 --warmup 3
