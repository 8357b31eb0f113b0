#!/bin/bash
# round 2, pass F: resident-weight convT forward + data gradient (LDS-staged stores, 6-deep
# ring): numerics, micro A/B against the GEMM kernels, flagship bench
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_unet_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for cfg in "0 6" "1 3" "1 6"; do
  set -- $cfg
  DDLPC_CONVT_RES=$1 DDLPC_CONVT_NBUF=$2 timeout -k 10 120 python -u scripts/conv_micro.py --batch 128 --passes tfwd,tdgrad > $O/micro_t_res$1_nb$2.txt 2>&1 || exit 1
  echo "== res=$1 nbuf=$2"; grep -v amdgpu.ids $O/micro_t_res$1_nb$2.txt
done
timeout -k 10 300 python -u bench.py --heartbeat 30 > $O/bench.json 2> $O/bench.err || exit 1
python scripts/summ_bench.py $O/bench.json
