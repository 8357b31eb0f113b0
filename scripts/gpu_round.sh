#!/bin/bash
# One GPU-box pass: GPU tests, smoke, benches (eager + hipGraph), rocprofv3 kernel stats.
# Every GPU step has its own time limit; the first failing step ends the script.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {   # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  tail -${TAIL:-15} gpurun_out/$name.log
  if [ $rc -ne 0 ]; then echo "!! $name rc=$rc"; exit $rc; fi
}
python scripts/build_ext.py > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
[ -z "$SKIP_TESTS" ] && step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --steps ${STEPS:-20} --warmup 5
step bench_graph 300 python bench.py --steps ${STEPS:-20} --warmup 5 --hip-graph 1
if [ -n "$PROF" ]; then
  step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py --batch 32 --steps 5 --warmup 2
  f=$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)
  python scripts/trace_summary.py "$f" 7 > gpurun_out/prof_summary.txt 2>&1
  head -45 gpurun_out/prof_summary.txt
fi
