# last sanity pass on the final tree: full GPU suite, smoke, headline bench
scripts/gpu.sh r6an \
 "tests:1000:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "bench:300:python -u bench.py"
