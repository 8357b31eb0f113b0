#!/bin/bash
# round 2, pass Y: paired 16-byte stores restricted to the variants where they measured faster:
# numerics, micro + bench A/B vs the 8-byte-store build, PMC of the 32-channel level-0 conv
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2y
mkdir -p $O
export TMPDIR=/tmp
OLD=$PWD/distributed-deep-learning-on-personal-computers_amd/_lib/ab/libddlpc_hip_b64.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "bn_backward_epilogue or dgrad or conv3_fwd or deferred" > $O/pytest_k.log 2>&1 || { tail -40 $O/pytest_k.log; exit 1; }
tail -2 $O/pytest_k.log
timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes fwd,dgrad,dgradbn > $O/micro_new.txt 2>&1 || { tail -20 $O/micro_new.txt; exit 1; }
DDLPC_LIB_PATH=$OLD DDLPC_CONV_ILV=0 timeout -k 10 200 python -u scripts/conv_micro.py --batch 128 --passes fwd,dgrad,dgradbn > $O/micro_old.txt 2>&1 || { tail -20 $O/micro_old.txt; exit 1; }
tail -1 $O/micro_new.txt; tail -1 $O/micro_old.txt
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run bench_new 200 python -u bench.py
run bench_old 200 env DDLPC_LIB_PATH=$OLD DDLPC_CONV_ILV=0 python -u bench.py
run bench_newb 200 python -u bench.py
for L in enc1.b enc2.b; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_$L/p1 -o run -- python3 scripts/conv_micro.py --batch 128 --passes fwd,dgrad --iters 1 --only $L > $O/pmc_$L.p1.log 2>&1 || { tail -20 $O/pmc_$L.p1.log; exit 3; }
  python scripts/pmc_summary.py $(find $O/pmc_$L/p1 -name '*counter_collection.csv' | head -1) > $O/pmc_${L}_sq.txt
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$L/p2 -o run -- python3 scripts/conv_micro.py --batch 128 --passes fwd,dgrad --iters 1 --only $L > $O/pmc_$L.p2.log 2>&1 || { tail -20 $O/pmc_$L.p2.log; exit 4; }
  python scripts/pmc_summary.py $(find $O/pmc_$L/p2 -name '*counter_collection.csv' | head -1) --raw > $O/pmc_${L}_fetch.txt
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_$L/p3 -o run -- python3 scripts/conv_micro.py --batch 128 --passes fwd,dgrad --iters 1 --only $L > $O/pmc_$L.p3.log 2>&1 || { tail -20 $O/pmc_$L.p3.log; exit 5; }
  python scripts/pmc_summary.py $(find $O/pmc_$L/p3 -name '*counter_collection.csv' | head -1) --raw > $O/pmc_${L}_write.txt
  cat $O/pmc_${L}_sq.txt $O/pmc_${L}_fetch.txt $O/pmc_${L}_write.txt
done
