#!/bin/bash
# round 2 session 2, pass G: packed-f32 head kernels, wgrad v3 on 8x8 layers by default:
# numerics (kernels + engine), bench x2, serial trace (head kernel times)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "head or wgrad" > $O/pytest_k.log 2>&1 || { tail -40 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_unet_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run bench_a 200 python -u bench.py
run bench_b 200 python -u bench.py
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 5 --warmup 3 --schedule serial > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 4; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python scripts/trace_summary.py "$f" 7 > $O/prof_summary.txt 2>&1; python scripts/stream_summary.py "$f" >> $O/prof_summary.txt 2>&1
python scripts/trace_summary.py "$f" 7 v | grep -E "head_" >> $O/prof_summary.txt
tail -8 $O/prof_summary.txt
