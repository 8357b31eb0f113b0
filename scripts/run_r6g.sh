OLD=distributed-deep-learning-on-personal-computers_amd/_lib/abtmp/libddlpc_hip_old.so
scripts/gpu.sh r6g \
 "tk:400:python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k 'head'" \
 "hm_new:120:python -u scripts/head_micro.py --batch 256" \
 "hm_old:120:DDLPC_LIB_PATH=$OLD python -u scripts/head_micro.py --batch 256" \
 "b_new1:200:python -u bench.py --steps 20 --warmup 5" \
 "b_old1:200:DDLPC_LIB_PATH=$OLD python -u bench.py --steps 20 --warmup 5" \
 "b_new2:200:python -u bench.py --steps 20 --warmup 5" \
 "b_old2:200:DDLPC_LIB_PATH=$OLD python -u bench.py --steps 20 --warmup 5" \
 "tu:600:python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_unet_gpu.py tests/test_data_gpu.py"
