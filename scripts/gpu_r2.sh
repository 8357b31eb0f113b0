#!/bin/bash
# Round-2 GPU pass: full GPU test suite, the driver bench, and the real train() entry point
# at bench batch (device-fed input pipeline) so the two throughputs can be compared.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TESTS:-tests}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -45 gpurun_out/pytest_gpu.log
# assertion failures (rc 1) do not stop the pass; crashes / timeouts do
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
[ -n "$NOBENCH" ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 3; }
cat gpurun_out/bench.json
timeout -k 10 300 python -u -m ddlpc train --impl hip --batch-per-gpu 128 --num-samples 12800 \
  --test-holdout 256 --max-steps 60 --log-every 10 --log-dir gpurun_out/train_b128 \
  > gpurun_out/train.json 2> gpurun_out/train.err || { tail -20 gpurun_out/train.err; exit 4; }
cat gpurun_out/train.json
grep images_per_s gpurun_out/train_b128/metrics.jsonl | cut -c1-220
exit $rc
