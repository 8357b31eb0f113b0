#!/bin/bash
# final check of the committed tree: GPU suite, smoke, bench
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s3c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 200 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 3; }
cat $O/bench.json
