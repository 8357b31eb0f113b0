#!/bin/bash
# source A/B on one box: micro with the tree as is (A), then with the files in $ALT_DIR
# copied over csrc/ (B).  The box's copy of the repo is scratch, so overwriting is fine.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
ALT_DIR=${ALT_DIR:-build/alt}
python scripts/build_ext.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 300 python scripts/conv_micro.py --iters ${ITERS:-20} --passes ${PASSES:-fwd,dgrad} $MICRO_ARGS > gpurun_out/micro_a.txt 2>&1 || { tail -20 gpurun_out/micro_a.txt; exit 3; }
mkdir -p /tmp/ab2_save && for f in $ALT_DIR/*; do cp csrc/$(basename $f) /tmp/ab2_save/; done
cp $ALT_DIR/* csrc/
python scripts/build_ext.py > gpurun_out/build_b.log 2>&1 || { cat gpurun_out/build_b.log; exit 1; }
timeout -k 10 300 python scripts/conv_micro.py --iters ${ITERS:-20} --passes ${PASSES:-fwd,dgrad} $MICRO_ARGS > gpurun_out/micro_b.txt 2>&1 || { tail -20 gpurun_out/micro_b.txt; exit 4; }
cp /tmp/ab2_save/* csrc/ && python scripts/build_ext.py > gpurun_out/build_c.log 2>&1
paste gpurun_out/micro_a.txt gpurun_out/micro_b.txt | grep -v amdgpu.ids
