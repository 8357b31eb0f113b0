set -e
o=gpurun_out/r6q
mkdir -p $o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $o/bench_default.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $o/bench_default2.log 2>&1
timeout -k 10 400 python -u bench.py --dims 3 --tile 128 --batch 8 --steps 10 --warmup 3 > $o/bench_3d.log 2>&1
timeout -k 10 400 python -u bench.py --tile 512 --batch 1 --accum 50 --steps 3 --warmup 2 > $o/bench_t512.log 2>&1
