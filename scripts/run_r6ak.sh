# CPU kernel set: the GPU suite (incl. the CPU-vs-GPU engine test), smoke, headline bench
scripts/gpu.sh r6ak \
 "xdev:300:python -u -m pytest tests/test_engine_cpu.py -m gpu -x -v --timeout 200 --timeout-method thread" \
 "tests:1000:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "bench:300:python -u bench.py"
