#!/bin/bash
# round 2 session 2, pass F: head stats pass with 2-pixel load batches; weight gradient v3 on
# the 8x8 bottleneck layers (DDLPC_WGRAD_MINW=8): numerics, micro, bench A/B, serial trace
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "head" > $O/pytest_k.log 2>&1 || { tail -40 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
DDLPC_WGRAD_MINW=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" > $O/pytest_w.log 2>&1 || { tail -40 $O/pytest_w.log; exit 1; }
tail -1 $O/pytest_w.log
timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes wgrad --only mid > $O/micro_w16.txt 2>&1 || { tail -20 $O/micro_w16.txt; exit 1; }
DDLPC_WGRAD_MINW=8 timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes wgrad --only mid > $O/micro_w8.txt 2>&1 || { tail -20 $O/micro_w8.txt; exit 1; }
cat $O/micro_w16.txt $O/micro_w8.txt
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run bench_a 200 python -u bench.py
run bench_w8 200 env DDLPC_WGRAD_MINW=8 python -u bench.py
run bench_b 200 python -u bench.py
run bench_w8b 200 env DDLPC_WGRAD_MINW=8 python -u bench.py
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 5 --warmup 3 --schedule serial > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 4; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python scripts/trace_summary.py "$f" 7 > $O/prof_summary.txt 2>&1; python scripts/stream_summary.py "$f" >> $O/prof_summary.txt 2>&1
python scripts/trace_summary.py "$f" 7 v | grep -E "head_" >> $O/prof_summary.txt
tail -8 $O/prof_summary.txt
