#!/bin/bash
# round 2 session 2, pass H: packed-f32 head kernels + fused 64-channel transposed-conv
# backward: numerics (kernels + engine), micro, bench A/B, serial trace
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/s2h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "head or wgrad or convt or deferred" > $O/pytest_k.log 2>&1 || { tail -40 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_unet_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes tbwdf,tbwds --only up1 > $O/micro.txt 2>&1 || { tail -20 $O/micro.txt; exit 1; }
cat $O/micro.txt
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run bench_f1 200 python -u bench.py
run bench_f0 200 env DDLPC_CONVT_FUSED=0 python -u bench.py
run bench_f1b 200 python -u bench.py
run bench_f0b 200 env DDLPC_CONVT_FUSED=0 python -u bench.py
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 5 --warmup 3 --schedule serial > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 4; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python scripts/trace_summary.py "$f" 7 > $O/prof_summary.txt 2>&1; python scripts/stream_summary.py "$f" >> $O/prof_summary.txt 2>&1
python scripts/trace_summary.py "$f" 7 v | grep -E "head_|convt_|gemm_tn" >> $O/prof_summary.txt
tail -14 $O/prof_summary.txt
