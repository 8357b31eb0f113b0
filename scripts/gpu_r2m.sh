#!/bin/bash
# round 2, pass M: fragment double buffering in the streaming conv: numerics, per-layer A/B,
# bench A/B (same box)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv3 or concat or split or res or fwd" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 0 1; do
  DDLPC_CONV_FDB=$v timeout -k 10 150 python -u scripts/conv_micro.py --batch 128 --passes fwd,dgrad > $O/micro_fdb$v.txt 2>&1 || exit 1
done
paste <(grep -v amdgpu $O/micro_fdb0.txt | cut -c1-40) <(grep -v amdgpu $O/micro_fdb1.txt | cut -c16-40)
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run bench_fdb1 200 python -u bench.py
run bench_fdb0 200 env DDLPC_CONV_FDB=0 python -u bench.py
run bench_fdb1b 200 python -u bench.py
