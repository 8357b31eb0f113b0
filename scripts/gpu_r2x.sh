#!/bin/bash
# round 2, pass X: 16-byte paired epilogue stores (pair16) in the conv kernels: numerics,
# per-layer micro A/B against the 8-byte-store build, bench A/B, serial trace
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2x
mkdir -p $O
export TMPDIR=/tmp
OLD=$PWD/distributed-deep-learning-on-personal-computers_amd/_lib/ab/libddlpc_hip_b64.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "bn_backward_epilogue or dgrad or conv3_fwd or deferred" > $O/pytest_k.log 2>&1 || { tail -40 $O/pytest_k.log; exit 1; }
tail -2 $O/pytest_k.log
timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes fwd,dgrad,dgradbn > $O/micro_new.txt 2>&1 || { tail -20 $O/micro_new.txt; exit 1; }
tail -1 $O/micro_new.txt
DDLPC_LIB_PATH=$OLD DDLPC_CONV_ILV=0 timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes fwd,dgrad,dgradbn > $O/micro_old.txt 2>&1 || { tail -20 $O/micro_old.txt; exit 1; }
tail -1 $O/micro_old.txt
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run bench_new 200 python -u bench.py
run bench_old 200 env DDLPC_LIB_PATH=$OLD DDLPC_CONV_ILV=0 python -u bench.py
run bench_newb 200 python -u bench.py
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_unet_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --schedule serial > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
echo prof done
