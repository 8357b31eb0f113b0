#!/bin/bash
# round 2 session 2, pass L: head forward fused with the backward statistics pass:
# numerics (kernels + engine), bench A/B, serial trace of the head kernels
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "head" > $O/pytest_k.log 2>&1 || { tail -40 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_unet_gpu.py tests/test_data_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json | cut -c1-220; [ $rc -eq 0 ] || exit $rc; }
run bench_f1 200 python -u bench.py
run bench_f0 200 env DDLPC_HEAD_FUSED_FWD=0 python -u bench.py
run bench_f1b 200 python -u bench.py
run bench_f0b 200 env DDLPC_HEAD_FUSED_FWD=0 python -u bench.py
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 5 --warmup 3 --schedule serial > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 4; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python scripts/trace_summary.py "$f" 7 > $O/prof_summary.txt 2>&1; python scripts/stream_summary.py "$f" >> $O/prof_summary.txt 2>&1
python scripts/trace_summary.py "$f" 7 v | grep -E "head_|ce_final" >> $O/prof_summary.txt
tail -8 $O/prof_summary.txt
