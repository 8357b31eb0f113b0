#!/bin/bash
# round 2, pass T: activation recompute (test, 1024^2 x 128 / 256 memory + speed), kernel
# traces of 1024^2 at batch 32 and 64 (serial) for the per-image scaling comparison
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_unet_gpu.py -k "recompute" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.json 2> $O/$name.err; local rc=$?; echo "== $name rc=$rc"; python scripts/summ_bench.py $O/$name.json; [ $rc -eq 0 ] || exit $rc; }
run t1024_b128_rc2 400 python -u bench.py --tile 1024 --batch 128 --steps 3 --warmup 2 --recompute 2 --heartbeat 30
run t1024_b256_rc2 600 python -u bench.py --tile 1024 --batch 256 --steps 2 --warmup 2 --recompute 2 --schedule serial --heartbeat 30
for b in 32 64; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof$b -o run -- python3 $GRAFT_REPO_ROOT/bench.py --tile 1024 --batch $b --steps 3 --warmup 2 --schedule serial > $GRAFT_REPO_ROOT/$O/prof$b.log 2>&1 || exit 1
  cd $GRAFT_REPO_ROOT
  echo prof $b done
done
