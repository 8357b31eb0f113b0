#!/bin/bash
# round 2, pass I: no host sync in the input path (device indices), lag-bounded side stream
# at 1024^2 x 128, GPU tests of the touched paths, profiles
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_data_gpu.py tests/test_unet_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to python -u bench.py --heartbeat 30 "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run flag_render 200
run flag_fixed 200 --fixed-batch 1
run flag_render2 200
run t1024_b128 400 --tile 1024 --batch 128 --steps 3 --warmup 3
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --schedule overlap > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
echo prof done
