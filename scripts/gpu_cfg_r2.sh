#!/bin/bash
# BASELINE.json configs #4 / #5 and the standard-width model on the HIP path (CFG=hip) or the
# in-house stock-PyTorch (MIOpen) baselines for the same shapes (CFG=torch).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/configs
export TMPDIR=/tmp
run() {   # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python -u bench.py --heartbeat 30 "$@" > gpurun_out/configs/$name.json 2> gpurun_out/configs/$name.err
  local rc=$?
  echo "== $name rc=$rc"; cut -c1-400 gpurun_out/configs/$name.json; [ $rc -ne 0 ] && tail -3 gpurun_out/configs/$name.err
  case $rc in 0|1|2) ;; *) echo "fatal rc=$rc, stopping"; exit $rc;; esac
  return 0
}
if [ "$CFG" = "hip" ]; then
  run t1024_b32 240 --tile 1024 --batch 32 --steps 5 --warmup 3
  run t1024_b64 240 --tile 1024 --batch 64 --steps 4 --warmup 3
  run t1024_b128 300 --tile 1024 --batch 128 --steps 3 --warmup 3
  run d3_128_b8 240 --dims 3 --tile 128 --batch 8 --steps 5 --warmup 3
  run wd1_b32 200 --width-divisor 1 --batch 32 --steps 10 --warmup 3
  run wd1_b64 200 --width-divisor 1 --batch 64 --steps 10 --warmup 3
elif [ "$CFG" = "torch_d3" ]; then     # stock PyTorch; MIOpen's exhaustive 3-D search did not finish
  # in 15 min (and logged missing CK instances), so FAST find mode (its heuristic choice)
  MIOPEN_FIND_MODE=FAST run d3_128_b8_torch 900 --impl torch --dims 3 --tile 128 --batch 8 --steps 5 --warmup 3
elif [ "$CFG" = "torch_wd1" ]; then
  MIOPEN_FIND_MODE=FAST run wd1_b64_torch 900 --impl torch --width-divisor 1 --batch 64 --steps 10 --warmup 3
fi
