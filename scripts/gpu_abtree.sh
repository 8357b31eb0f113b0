#!/bin/bash
# Same-box A/B of whole source files: A = the tree as sent, B = the files mirrored under
# $ALT (paths relative to the repo root).  Runs A B A B so box drift shows up.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
ALT=${ALT:-build/alttree}
files=$(cd $ALT && find . -type f | sed 's#^\./##')
mkdir -p /tmp/abA && for f in $files; do mkdir -p /tmp/abA/$(dirname $f); cp $f /tmp/abA/$f; done
run() {   # tag
  python scripts/build_ext.py > gpurun_out/ab/build_$1.log 2>&1 || { tail -20 gpurun_out/ab/build_$1.log; exit 1; }
  timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 5 $BENCH_ARGS > gpurun_out/ab/$1.json 2> gpurun_out/ab/$1.err || { tail -5 gpurun_out/ab/$1.err; exit 2; }
  echo "$1 $(python -c "import json; r=json.load(open('gpurun_out/ab/$1.json')); print(r['value'], r['ms_per_step'])")"
}
useA() { for f in $files; do cp /tmp/abA/$f $f; done; }
useB() { for f in $files; do cp $ALT/$f $f; done; }
run A1; useB; run B1; useA; run A2; useB; run B2; useA
