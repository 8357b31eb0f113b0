#!/bin/bash
# single-GPU step as one hipGraph replay vs eager launches, on the current kernel mix
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s3b
mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json | cut -c1-100; [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }; }
run eager1 200 python -u bench.py
run graph1 240 python -u bench.py --hip-graph 1
run eager2 200 python -u bench.py
run graph2 240 python -u bench.py --hip-graph 1
