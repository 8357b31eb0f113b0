# final-tree validation after the CPU kernel set: GPU suite, smoke, headline x2, every BASELINE configuration, trace
scripts/gpu.sh r6final3 \
 "tests:1000:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "bench:300:python -u bench.py" \
 "bench2:300:python -u bench.py --steps 20 --warmup 5" \
 "b_t512:300:python -u bench.py --tile 512 --batch 1 --accum 50 --steps 4 --warmup 2" \
 "b_3d:300:python -u bench.py --dims 3 --tile 128 --batch 8 --steps 10 --warmup 5" \
 "b_wd1:300:python -u bench.py --width-divisor 1 --batch 64 --steps 10 --warmup 5" \
 "b_1024:400:python -u bench.py --tile 1024 --batch 32 --steps 5 --warmup 3" \
 "b_b256:300:python -u bench.py --batch 256 --steps 20 --warmup 5" \
 "prof:400:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6final3/prof -o run -- python3 bench.py --steps 5 --warmup 3 --schedule serial"
