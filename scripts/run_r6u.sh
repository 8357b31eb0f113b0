# validation after the late-epilogue and 256-column convT changes; serial trace at batch 384
scripts/gpu.sh r6u \
 "tests:1000:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
 "bench:300:python -u bench.py" \
 "bench2:300:python -u bench.py --steps 20 --warmup 5" \
 "b_t512:300:python -u bench.py --tile 512 --batch 1 --accum 50 --steps 4 --warmup 2" \
 "b_3d:300:python -u bench.py --dims 3 --tile 128 --batch 8 --steps 10 --warmup 5" \
 "prof:400:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6u/prof -o run -- python3 bench.py --steps 5 --warmup 3 --schedule serial"
