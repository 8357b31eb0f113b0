#!/bin/bash
# round 2 session 2, pass X: full re-check after the launch-count changes (convT data-gradient
# BN partials without the zero-fill pass, head gradient scale and meter as single launches)
# — GPU suite, smoke, bench x2, serial kernel trace (step summary)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json | cut -c1-160; [ $rc -eq 0 ] || exit $rc; }
run bench1 200 python -u bench.py
run bench2 200 python -u bench.py
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 5 --warmup 3 --schedule serial > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 4; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python scripts/trace_summary.py "$f" 7 > $O/prof_summary.txt 2>&1; python scripts/stream_summary.py "$f" >> $O/prof_summary.txt 2>&1
head -4 $O/prof_summary.txt
