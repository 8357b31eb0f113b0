# CPU kernel set, third pass: the CPU-vs-GPU engine test (cosine report), GPU suite, smoke, bench
scripts/gpu.sh r6am \
 "xdev:300:python -u -m pytest tests/test_engine_cpu.py -m gpu -v -s --timeout 200 --timeout-method thread" \
 "tests:1000:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "bench:300:python -u bench.py"
