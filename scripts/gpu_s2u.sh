#!/bin/bash
# round 2 session 2, pass U: SQ counters of the largest kernel classes for the next round's
# planning — streaming 3x3 conv (enc3.b / dec3.a fwd + dgrad), resident conv + v3 weight
# gradient at 256^2 (dec1.a), v2 concat weight gradient (dec2.a), deep v3 wgrad (enc4.b)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2u
mkdir -p $O
export TMPDIR=/tmp
for spec in enc3.b:fwd,dgrad dec3.a:fwd,dgrad dec1.a:fwd,dgrad,wgrad dec2.a:wgrad enc4.b:wgrad; do
  L=${spec%%:*}; P=${spec#*:}
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/$L -o run -- python3 scripts/conv_micro.py --batch 128 --passes $P --iters 1 --only $L > $O/$L.log 2>&1 || { tail -20 $O/$L.log; exit 3; }
  f=$(find $O/$L -name '*counter_collection.csv' | head -1)
  echo "== $L ($P)"; python scripts/pmc_summary.py "$f" | tee $O/${L}_sq.txt
done
