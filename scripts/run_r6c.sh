scripts/gpu.sh r6c \
 "tk:300:python -u -m pytest -x -v --timeout 200 --timeout-method thread -s tests/test_kernels_gpu.py -k 'c32'" \
 "on1:200:python -u bench.py --steps 20 --warmup 5" \
 "off1:200:python -u bench.py --steps 20 --warmup 5 --engine-set c32_bnp=0" \
 "on2:200:python -u bench.py --steps 20 --warmup 5" \
 "off2:200:python -u bench.py --steps 20 --warmup 5 --engine-set c32_bnp=0" \
 "tu:600:python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_unet_gpu.py"
