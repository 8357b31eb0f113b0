#!/bin/bash
# streaming / resident 3x3 conv knobs re-checked on the final build (conv_micro fwd + dgrad,
# all 22 layers at batch 128; default bracketing the variants)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s3d
mkdir -p $O
export TMPDIR=/tmp
m() { local name=$1; shift; timeout -k 10 150 env "$@" python -u scripts/conv_micro.py --batch 128 --passes fwd,dgrad > $O/$name.txt 2>&1 || { tail -20 $O/$name.txt; exit 2; }; echo "== $name: $(tail -1 $O/$name.txt | cut -c1-150)"; }
m def_a DDLPC_X=0
m nbb3 DDLPC_CONV_NBB=3
m super0 DDLPC_CONV_SUPER=0
m fdb0 DDLPC_CONV_FDB=0
m ilv1 DDLPC_CONV_ILV=1
m cfg4_0 DDLPC_CONV_CFG4=0
m resdepth2 DDLPC_RES_DEPTH=2
m def_b DDLPC_X=0
