#!/bin/bash
# round 2, pass R: 32x32x16 weight-gradient kernel (v3): numerics, per-layer A/B vs v2,
# bank-conflict PMC on the 32-channel layers, bench A/B
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" tests/test_unet_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 0 1; do
  DDLPC_WGRAD_V3=$v timeout -k 10 150 python -u scripts/conv_micro.py --batch 128 --passes wgrad > $O/micro_v3_$v.txt 2>&1 || exit 1
done
paste <(grep -v amdgpu $O/micro_v3_0.txt | cut -c1-40) <(grep -v amdgpu $O/micro_v3_1.txt | cut -c16-40)
cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc -o run -- python3 $GRAFT_REPO_ROOT/scripts/conv_micro.py --batch 128 --passes wgrad --iters 1 --only 1.b > $GRAFT_REPO_ROOT/$O/pmc.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/pmc.log; exit 3; }
cd $GRAFT_REPO_ROOT
f=$(find $O/pmc -name '*counter_collection.csv' | head -1)
python scripts/pmc_summary.py "$f" | tee $O/pmc_summary.txt
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run bench_v3 200 python -u bench.py
run bench_v2 200 env DDLPC_WGRAD_V3=0 python -u bench.py
run bench_v3b 200 python -u bench.py
