#!/bin/bash
# round 2 session 2, pass N: head kernels with DPP lane sums, fast reciprocal and packed
# accumulators: numerics, micro + bench A/B against the previous build, SQ counters
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${PASS:-s2n}
mkdir -p $O
export TMPDIR=/tmp
OLD=$PWD/distributed-deep-learning-on-personal-computers_amd/_lib/ab/libddlpc_hip_${OLDLIB:-headdpp}.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "head" > $O/pytest_k.log 2>&1 || { tail -40 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
timeout -k 10 120 python -u scripts/head_micro.py > $O/micro_new.txt 2>&1 || { tail -20 $O/micro_new.txt; exit 2; }
DDLPC_LIB_PATH=$OLD timeout -k 10 120 python -u scripts/head_micro.py > $O/micro_old.txt 2>&1 || { tail -20 $O/micro_old.txt; exit 2; }
timeout -k 10 120 python -u scripts/head_micro.py > $O/micro_new2.txt 2>&1 || { tail -20 $O/micro_new2.txt; exit 2; }
echo new; cat $O/micro_new.txt; echo old; cat $O/micro_old.txt; echo new2; cat $O/micro_new2.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d $O/pmc1 -o run -- python3 scripts/head_micro.py --iters 1 > $O/pmc1.log 2>&1 || { tail -20 $O/pmc1.log; exit 3; }
python scripts/pmc_summary.py $(find $O/pmc1 -name '*counter_collection.csv' | head -1) > $O/pmc_sq.txt
cat $O/pmc_sq.txt
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json | cut -c1-120; [ $rc -eq 0 ] || exit $rc; }
run new 200 python -u bench.py
run old 200 env DDLPC_LIB_PATH=$OLD python -u bench.py
run newb 200 python -u bench.py
run oldb 200 env DDLPC_LIB_PATH=$OLD python -u bench.py
