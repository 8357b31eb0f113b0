#!/bin/bash
# round 2, pass H: DP GPU tests (codec / accumulation / bf16 wire), fixed-batch vs per-step
# input diagnostic, config #4 at batch 64 / 128 with the alternating schedule probe
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_dp_gpu.py > $O/pytest_dp.log 2>&1 || { tail -40 $O/pytest_dp.log; exit 1; }
tail -3 $O/pytest_dp.log
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to python -u bench.py --heartbeat 30 "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run flag_fixed 200 --fixed-batch 1
run flag_render 200
run flag_fixed2 200 --fixed-batch 1
run flag_render2 200
run t1024_b64 300 --tile 1024 --batch 64 --steps 4 --warmup 3
run t1024_b128 400 --tile 1024 --batch 128 --steps 3 --warmup 3
