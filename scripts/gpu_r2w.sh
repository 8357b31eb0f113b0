#!/bin/bash
# round 2, pass W: super-stage conv with the next stage's DMAs interleaved between the MFMAs
# (ILV): numerics, per-layer micro A/B, bench A/B
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "bn_backward_epilogue or dgrad or conv3_fwd" > $O/pytest_k.log 2>&1 || { tail -40 $O/pytest_k.log; exit 1; }
tail -2 $O/pytest_k.log
for v in 1 0; do
  DDLPC_CONV_ILV=$v timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes fwd,dgrad,dgradbn > $O/micro_ilv$v.txt 2>&1 || { tail -20 $O/micro_ilv$v.txt; exit 1; }
  tail -1 $O/micro_ilv$v.txt
done
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run bench_ilv1 200 python -u bench.py
run bench_ilv0 200 env DDLPC_CONV_ILV=0 python -u bench.py
run bench_ilv1b 200 python -u bench.py
