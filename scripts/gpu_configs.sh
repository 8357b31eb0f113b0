#!/bin/bash
# BASELINE.json configs: batch sweep (HIP vs stock PyTorch/MIOpen), 1024^2 tiles, 3-D 128^3.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/configs
export TMPDIR=/tmp
python scripts/build_ext.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
run() {   # name, args...
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/configs/$name.json 2> gpurun_out/configs/$name.err
  local rc=$?
  echo "== $name rc=$rc"; cat gpurun_out/configs/$name.json; [ $rc -ne 0 ] && tail -3 gpurun_out/configs/$name.err
  case $rc in 124|134|137|139) echo "fatal rc=$rc, stopping"; exit $rc;; esac
  return 0
}
for spec in $CONFIGS; do
  IFS=: read -r name argstr <<< "$spec"
  run $name ${argstr//,/ }
done
