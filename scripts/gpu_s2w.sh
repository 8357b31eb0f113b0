#!/bin/bash
# round 2 session 2, pass W: does the ~4.5 us floor of every small kernel in the step trace
# move with kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1)?  bench A/B/A/B;
# plus the head gradient-scale op (one launch instead of five elementwise kernels)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2w
mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json | cut -c1-100; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "head or meter" tests/test_unet_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run def1 200 python -u bench.py
run dk1 200 env HIP_FORCE_DEV_KERNARG=1 python -u bench.py
run def2 200 python -u bench.py
run dk2 200 env HIP_FORCE_DEV_KERNARG=1 python -u bench.py
