#!/bin/bash
# secondary configs re-measured on the final tree (config #4 1024^2, config #5 3-D 128^3,
# standard-width U-Net) and the train() entry point against bench.py on the same box
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s3e
mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json | cut -c1-90; [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }; }
run bench 200 python -u bench.py
run t1024_b32 240 python -u bench.py --tile 1024 --batch 32 --steps 5 --warmup 3
run t1024_b128 400 python -u bench.py --tile 1024 --batch 128 --steps 3 --warmup 3
run d3_128_b8 240 python -u bench.py --dims 3 --tile 128 --batch 8 --steps 5 --warmup 3
run wd1_b64 200 python -u bench.py --width-divisor 1 --batch 64 --steps 10 --warmup 3
