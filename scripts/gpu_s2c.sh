#!/bin/bash
# round 2 session 2, pass C: transposed-conv weight gradient v2 (64x64 wave tiles, LDS-DMA):
# numerics, micro A/B vs v1, engine tests, bench A/B
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "convt or deferred or out_params" > $O/pytest_k.log 2>&1 || { tail -40 $O/pytest_k.log; exit 1; }
tail -2 $O/pytest_k.log
timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes twgrad,tfwd,tdgrad > $O/micro_v2.txt 2>&1 || { tail -20 $O/micro_v2.txt; exit 1; }
DDLPC_CONVT_WG2=0 timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes twgrad > $O/micro_v1.txt 2>&1 || { tail -20 $O/micro_v1.txt; exit 1; }
cat $O/micro_v2.txt $O/micro_v1.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_unet_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run bench_w2 200 python -u bench.py
run bench_w1 200 env DDLPC_CONVT_WG2=0 python -u bench.py
run bench_w2b 200 python -u bench.py
run bench_w1b 200 env DDLPC_CONVT_WG2=0 python -u bench.py
