#!/bin/bash
# round 2, pass G: convT resident kernels (occupancy-gated planner, 3-deep ring, LDS-DMA y prefetch)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "convt or deferred" tests/test_unet_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for v in 0 1; do
  DDLPC_CONVT_RES=$v timeout -k 10 120 python -u scripts/conv_micro.py --batch 128 --passes tfwd,tfwdbn,tdgrad,tdgradbn > $O/micro_t_res$v.txt 2>&1 || exit 1
  echo "== res=$v"; grep -v amdgpu.ids $O/micro_t_res$v.txt
done
timeout -k 10 300 python -u bench.py --heartbeat 30 > $O/bench.json 2> $O/bench.err || exit 1
python scripts/summ_bench.py $O/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --schedule serial > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
echo prof done
