# final-tree validation after the last kernel changes: GPU suite, smoke, headline x2, serial-schedule kernel trace
scripts/gpu.sh r6final2 \
 "tests:1000:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "bench:300:python -u bench.py" \
 "bench2:300:python -u bench.py --steps 20 --warmup 5" \
 "prof:400:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6final2/prof -o run -- python3 bench.py --steps 5 --warmup 3 --schedule serial"
