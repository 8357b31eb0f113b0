#!/bin/bash
# round 2 session 2, pass Q: weight gradient v3 with a 3-deep DMA ring (32-channel layers,
# 128-pixel tiles): numerics, per-layer micro A/B, bench A/B
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2q
mkdir -p $O
export TMPDIR=/tmp
DDLPC_WGRAD3_RING=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" > $O/pytest_k.log 2>&1 || { tail -40 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes wgrad > $O/micro_r0.txt 2>&1 || { tail -20 $O/micro_r0.txt; exit 2; }
DDLPC_WGRAD3_RING=1 timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes wgrad > $O/micro_r1.txt 2>&1 || { tail -20 $O/micro_r1.txt; exit 2; }
grep -E "enc1|dec1|totals" $O/micro_r0.txt; grep -E "enc1|dec1|totals" $O/micro_r1.txt
DDLPC_WGRAD3_RING=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_unet_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
run r1 200 env DDLPC_WGRAD3_RING=1 python -u bench.py
run r0 200 python -u bench.py
run r1b 200 env DDLPC_WGRAD3_RING=1 python -u bench.py
run r0b 200 python -u bench.py
