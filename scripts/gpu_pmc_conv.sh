#!/bin/bash
# 3x3 conv forward / data-gradient PMC passes on one layer (ONLY=<name>, PASSES=fwd,dgrad):
# pass 1 SQ (MFMA busy, waits, LDS), pass 2 TCC (L2 hit/miss), pass 3 TA/TD busy
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/pmc_conv_${ONLY:-enc4.b}
mkdir -p $O
export TMPDIR=/tmp
P=${PASSES:-fwd,dgrad}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 scripts/conv_micro.py --batch 128 --passes $P --iters 1 --only ${ONLY:-enc4.b} > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 3; }
f=$(find $O/p1 -name '*counter_collection.csv' | head -1)
python scripts/pmc_summary.py "$f" | tee $O/p1_summary.txt
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d $O/p2 -o run -- python3 scripts/conv_micro.py --batch 128 --passes $P --iters 1 --only ${ONLY:-enc4.b} > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 4; }
f=$(find $O/p2 -name '*counter_collection.csv' | head -1)
python scripts/pmc_summary.py "$f" --raw | tee $O/p2_summary.txt
