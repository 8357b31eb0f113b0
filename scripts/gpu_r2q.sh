#!/bin/bash
# round 2, pass Q: super-stages (two kernel rows per barrier) in the 8-wave streaming conv:
# numerics, per-layer A/B, bench A/B on one box
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_unet_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 0 1; do
  DDLPC_CONV_SUPER=$v timeout -k 10 150 python -u scripts/conv_micro.py --batch 128 --passes fwd,dgrad > $O/micro_super$v.txt 2>&1 || exit 1
done
paste <(grep -v amdgpu $O/micro_super0.txt | cut -c1-40) <(grep -v amdgpu $O/micro_super1.txt | cut -c16-40)
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run bench_super1 200 python -u bench.py
run bench_super0 200 env DDLPC_CONV_SUPER=0 python -u bench.py
run bench_super1b 200 python -u bench.py
