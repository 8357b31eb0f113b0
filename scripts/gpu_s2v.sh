#!/bin/bash
# round 2 session 2, pass V: weight-gradient v2 LDS bank conflicts (dec2.a showed
# 2.9e7 conflict cycles after the dY-prologue table was added) — tile buffers 1-KiB aligned
# vs the HEAD build: SQ counters + per-layer timing
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2v
mkdir -p $O
export TMPDIR=/tmp
OLD=$PWD/distributed-deep-learning-on-personal-computers_amd/_lib/ab/libddlpc_hip_head.so
pmc() { local tag=$1 L=$2
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/${tag}_$L -o run -- python3 scripts/conv_micro.py --batch 128 --passes wgrad --iters 1 --only $L > $O/${tag}_$L.log 2>&1 || { tail -20 $O/${tag}_$L.log; exit 3; }
  f=$(find $O/${tag}_$L -name '*counter_collection.csv' | head -1)
  echo "== $tag $L"; python scripts/pmc_summary.py "$f" | tee $O/${tag}_${L}_sq.txt
}
pmc new dec2.a && pmc new dec3.a && pmc new enc2.b
export DDLPC_LIB_PATH=$OLD
pmc old dec2.a && pmc old dec3.a
unset DDLPC_LIB_PATH
timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes wgrad > $O/micro_new.txt 2>&1 || { tail -20 $O/micro_new.txt; exit 2; }
DDLPC_LIB_PATH=$OLD timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes wgrad > $O/micro_old.txt 2>&1 || { tail -20 $O/micro_old.txt; exit 2; }
paste <(awk '{print $1, $3}' $O/micro_new.txt) <(awk '{print $3}' $O/micro_old.txt)
