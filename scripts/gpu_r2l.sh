#!/bin/bash
# round 2, pass L: PMC of the streaming 3x3 conv (8-wave config) on two mid layers
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
ONLY=enc4.b PASSES=fwd,dgrad bash scripts/gpu_pmc_conv.sh && ONLY=dec3.a PASSES=fwd bash scripts/gpu_pmc_conv.sh
