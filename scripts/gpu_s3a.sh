#!/bin/bash
# BN-backward apply pass (bn_bwd2 MODE 1, no pool): loads in flight per lane (2 vs 4) and
# streaming (nontemporal) dY stores — numerics with the variant, per-kernel time per variant
# (the DDLPC_BN_APPLY_U / _NT knobs were removed after this measurement: neither helped)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s3a
mkdir -p $O
export TMPDIR=/tmp
DDLPC_BN_APPLY_U=4 DDLPC_BN_APPLY_NT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "bn" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "2 0" "4 0" "2 1" "4 1"; do
  set -- $v
  DDLPC_BN_APPLY_U=$1 DDLPC_BN_APPLY_NT=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/u$1nt$2 -o run -- python3 scripts/bn_micro.py --iters 10 > $O/u$1nt$2.log 2>&1 || { tail -20 $O/u$1nt$2.log; exit 2; }
  f=$(find $O/u$1nt$2 -name '*kernel_stats.csv' | head -1)
  echo "== U=$1 NT=$2"; python - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "bn_bwd2_kernel<2, false, 1" in n:
        print(f'{n[n.find("bn_bwd2"):][:48]:48s} calls {r["Calls"]:>5s} total {float(r["TotalDurationNs"])/1e3:9.1f} us avg {float(r["AverageNs"])/1e3:7.2f} us')
PY
done
