#!/bin/bash
# bench.py under several environment settings on one box: ENVS="name:K=V,K=V name2:..."
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/envs
export TMPDIR=/tmp
python scripts/build_ext.py > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
for spec in $ENVS; do
  IFS=: read -r name kv <<< "$spec"
  envs=(${kv//,/ })
  env "${envs[@]}" timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 5 $BENCH_ARGS > gpurun_out/envs/$name.json 2> gpurun_out/envs/$name.err
  rc=$?
  echo "== $name ($kv) rc=$rc $(python -c "import json,sys; r=json.load(open('gpurun_out/envs/$name.json')); print(r['value'], r['ms_per_step'])" 2>/dev/null)"
  case $rc in 0) ;; *) tail -5 gpurun_out/envs/$name.err; exit $rc;; esac
done
