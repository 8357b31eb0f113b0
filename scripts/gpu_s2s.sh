#!/bin/bash
# round 2 session 2, pass S: weight gradient v3 after restoring the x_pix fast path —
# micro + bench A/B against the build before the ring commit, wgrad numerics
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2s
mkdir -p $O
export TMPDIR=/tmp
OLD=$PWD/distributed-deep-learning-on-personal-computers_amd/_lib/ab/libddlpc_hip_prering.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" > $O/pytest_k.log 2>&1 || { tail -40 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes wgrad > $O/micro_new.txt 2>&1 || { tail -20 $O/micro_new.txt; exit 2; }
DDLPC_LIB_PATH=$OLD timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes wgrad > $O/micro_old.txt 2>&1 || { tail -20 $O/micro_old.txt; exit 2; }
tail -1 $O/micro_new.txt; tail -1 $O/micro_old.txt
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
run new 200 python -u bench.py
run old 200 env DDLPC_LIB_PATH=$OLD python -u bench.py
run newb 200 python -u bench.py
run oldb 200 env DDLPC_LIB_PATH=$OLD python -u bench.py
