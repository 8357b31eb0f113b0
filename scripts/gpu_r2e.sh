#!/bin/bash
# round 2, pass E: resident-weight convT forward (tests + micro A/B) and the side-stream
# schedule at 1024^2 batch 64 (memory counters, allocator / priority variants)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r2e
export TMPDIR=/tmp
O=gpurun_out/r2e
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "convt or deferred" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for v in 0 1; do
  DDLPC_CONVT_RES=$v timeout -k 10 120 python -u scripts/conv_micro.py --batch 128 --passes tfwd > $O/micro_tfwd_res$v.txt 2>&1 || exit 1
  echo "== res=$v"; cat $O/micro_tfwd_res$v.txt
done
run() { local name=$1; shift; timeout -k 10 240 "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run side_b64 python -u bench.py --tile 1024 --batch 64 --steps 4 --warmup 3 --schedule overlap --heartbeat 30
run side_b64_prio0 env DDLPC_SIDE_PRIORITY=0 python -u bench.py --tile 1024 --batch 64 --steps 4 --warmup 3 --schedule overlap --heartbeat 30
run side_b64_exp env PYTORCH_HIP_ALLOC_CONF=expandable_segments:True python -u bench.py --tile 1024 --batch 64 --steps 4 --warmup 3 --schedule overlap --heartbeat 30
run flag_b128 python -u bench.py --heartbeat 30
