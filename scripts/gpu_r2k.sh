#!/bin/bash
# round 2, pass K: 3x3 streaming conv with a 3-deep weight ring (8-wave config) and fixed-count
# buffer-store epilogue: numerics, per-layer A/B against the double-buffered ring, bench
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_unet_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for v in 2 3; do
  DDLPC_CONV_NBB=$v timeout -k 10 150 python -u scripts/conv_micro.py --batch 128 --passes fwd,dgrad > $O/micro_nbb$v.txt 2>&1 || exit 1
  echo "== nbb=$v"; grep -v amdgpu.ids $O/micro_nbb$v.txt | tail -1
done
paste <(grep -v amdgpu $O/micro_nbb2.txt | cut -c1-40) <(grep -v amdgpu $O/micro_nbb3.txt | cut -c16-40)
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run bench_nbb3 200 python -u bench.py
run bench_nbb2 200 env DDLPC_CONV_NBB=2 python -u bench.py
run bench_nbb3b 200 python -u bench.py
