#!/bin/bash
# run bench.py N times (fresh processes) and print throughput + allocator counters
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/rep
export TMPDIR=/tmp
python scripts/build_ext.py > gpurun_out/build.log 2>&1 || exit 1
for i in $(seq 1 ${N:-8}); do
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 $BENCH_ARGS > gpurun_out/rep/$i.json 2> gpurun_out/rep/$i.err || { tail -3 gpurun_out/rep/$i.err; exit 2; }
  python -c "import json; r=json.load(open('gpurun_out/rep/$i.json')); c=r['config']; print($i, r['value'], r['ms_per_step'], c.get('schedule'), c.get('device_mallocs'))"
done
