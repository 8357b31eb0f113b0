#!/bin/bash
# round 2, pass P: one barrier per chunk-start stage (prologue before the barrier), padding-
# aware conv tile planner: numerics, per-layer times, bench
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_unet_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 150 python -u scripts/conv_micro.py --batch 128 --passes fwd,dgrad > $O/micro.txt 2>&1 || exit 1
grep -v amdgpu $O/micro.txt
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run bench1 200 python -u bench.py
run bench2 200 python -u bench.py
