#!/bin/bash
# round 2, pass U: deferred encoder skips (BN + ReLU applied by the decoder concat conv's X2
# prologue): numerics (kernel + engine), bench A/B, serial trace
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_unet_gpu.py tests/test_data_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run bench_dskip1 200 python -u bench.py
run bench_dskip0 200 env DDLPC_DEFER_SKIP=0 python -u bench.py
run bench_dskip1b 200 python -u bench.py
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --schedule serial > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
echo prof done
