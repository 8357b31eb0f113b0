#!/bin/bash
# round 2 session 2, final pass: GPU test suite, smoke, driver bench x2, train() entry point,
# BASELINE configs #4 (1024^2 b32, b128) / #5 (3-D 128^3 b8) / standard width b64
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json | cut -c1-140; [ $rc -eq 0 ] || exit $rc; }
run bench1 200 python -u bench.py
run bench2 200 python -u bench.py
timeout -k 10 300 python -u -m ddlpc train --impl hip --batch-per-gpu 128 --num-samples 12800 \
  --test-holdout 256 --max-steps 60 --log-every 10 --log-dir $O/train_b128 \
  > $O/train.json 2> $O/train.err || { tail -20 $O/train.err; exit 4; }
grep images_per_s $O/train_b128/metrics.jsonl | cut -c1-160 | tail -2
run t1024_b32 240 python -u bench.py --tile 1024 --batch 32 --steps 5 --warmup 3
run t1024_b128 400 python -u bench.py --tile 1024 --batch 128 --steps 3 --warmup 3
run d3_128_b8 240 python -u bench.py --dims 3 --tile 128 --batch 8 --steps 5 --warmup 3
run wd1_b64 200 python -u bench.py --width-divisor 1 --batch 64 --steps 10 --warmup 3
