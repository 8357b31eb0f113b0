#!/bin/bash
# One parametrised GPU-box runner (replaces the per-experiment gpu_*.sh scripts).
#
#   scripts/gpu.sh OUT STEP [STEP ...]
#
# OUT is a directory under gpurun_out/.  Each STEP is "name:timeout:command ..." (the command
# runs under `bash -c`, so it may quote: "t:300:pytest -k 'a or b'") or a shorthand below.  Every GPU step runs under its own
# `timeout -k 10`, writes OUT/name.log, and the first failing step ends the script (no GPU
# work after a fault, an abort or a time limit).
#
# shorthands:
#   tests           pytest -m gpu (one process, per-test thread timeout)
#   smoke           __graft_entry__.smoke()
#   bench           bench.py defaults (20 steps)
#   prof            rocprofv3 kernel trace of a batch-128 serial-schedule step + summary
#
# Extra bench runs: "b_NAME:TIMEOUT:python -u bench.py --tile 512 --batch 1 ..." — the JSON
# line lands in OUT/b_NAME.log.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:?usage: gpu.sh OUT STEP...}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
# the library built here travels with the snapshot: rebuild only if a source is newer
LIB=distributed-deep-learning-on-personal-computers_amd/_lib/libddlpc_hip.so
if [ -f "$LIB" ] && [ -z "$(find csrc -newer "$LIB" -type f | head -1)" ]; then
  echo "library up to date" > "$OUT/build.log"
else
  python scripts/build_ext.py > "$OUT/build.log" 2>&1 || { tail -30 "$OUT/build.log"; exit 1; }
fi

run_step() {   # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  tail -"${TAIL:-6}" "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "!! $name rc=$rc"; exit $rc; fi
}

for spec in "$@"; do
  case "$spec" in
    tests)
      run_step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf ;;
    smoke)
      run_step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      run_step bench 300 python -u bench.py ;;
    prof)
      run_step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
        python3 bench.py --steps 5 --warmup 3 --schedule serial
      f=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
      python scripts/trace_summary.py "$f" 5 > "$OUT/prof_summary.txt" 2>&1
      head -60 "$OUT/prof_summary.txt" ;;
    *:*:*)
      name=${spec%%:*}; rest=${spec#*:}; t=${rest%%:*}; cmd=${rest#*:}
      run_step "$name" "$t" bash -c "$cmd" ;;
    *)
      echo "unknown step: $spec"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
