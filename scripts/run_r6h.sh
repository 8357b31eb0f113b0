OLD=distributed-deep-learning-on-personal-computers_amd/_lib/abtmp/libddlpc_hip_old.so
scripts/gpu.sh r6h \
 "tk:400:python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k 'bn or pool or head'" \
 "bm_new:120:python -u scripts/bn_micro.py --batch 256" \
 "bm_old:120:DDLPC_LIB_PATH=$OLD python -u scripts/bn_micro.py --batch 256" \
 "b_new1:200:python -u bench.py --steps 20 --warmup 5" \
 "b_old1:200:DDLPC_LIB_PATH=$OLD python -u bench.py --steps 20 --warmup 5" \
 "b_new2:200:python -u bench.py --steps 20 --warmup 5" \
 "b_old2:200:DDLPC_LIB_PATH=$OLD python -u bench.py --steps 20 --warmup 5" \
 "d3_new:300:python -u bench.py --dims 3 --tile 128 --batch 8 --steps 10 --warmup 3" \
 "d3_old:300:DDLPC_LIB_PATH=$OLD python -u bench.py --dims 3 --tile 128 --batch 8 --steps 10 --warmup 3"
