#!/bin/bash
# round 2 session 2, pass A: fresh-container re-check — GPU tests, smoke, bench x2, b128 kernel trace
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py > $O/bench$i.json 2> $O/bench$i.err || { tail -20 $O/bench$i.err; exit 3; }
  python scripts/summ_bench.py $O/bench$i.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 5 --warmup 3 --schedule serial > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 4; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python scripts/trace_summary.py "$f" 7 > $O/prof_summary.txt 2>&1
python scripts/stream_summary.py "$f" >> $O/prof_summary.txt 2>&1
head -40 $O/prof_summary.txt
