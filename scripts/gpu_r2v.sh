#!/bin/bash
# round 2, pass V: BN1-backward reduction fused into the data-gradient epilogue (bnb):
# numerics (kernel + engine), micro A/B, bench A/B, serial trace
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "bn_backward_epilogue or dgrad or conv3_fwd" > $O/pytest_k.log 2>&1 || { tail -40 $O/pytest_k.log; exit 1; }
tail -2 $O/pytest_k.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_unet_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes dgrad,dgradbn --only .b > $O/micro.txt 2>&1 || { tail -20 $O/micro.txt; exit 1; }
cat $O/micro.txt
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run bench_bnb1 200 python -u bench.py
run bench_bnb0 200 env DDLPC_BNB_EPI=0 python -u bench.py
run bench_bnb1b 200 python -u bench.py
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --schedule serial > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
echo prof done
