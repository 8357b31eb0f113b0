# transposed-conv data gradient with 256-column tiles (new) vs HEAD: numerics, per level, bench
D=distributed-deep-learning-on-personal-computers_amd/_lib/diag
B="DDLPC_LIB_PATH=$D/libddlpc_diag_convt_gemm_HEAD.so"
scripts/gpu.sh r6w \
 "t:300:python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'convt or deferred_bn' --timeout 120 --timeout-method thread" \
 "ct_new:200:python -u scripts/conv_micro.py --batch 384 --passes tdgrad,tdgradbn --only up --iters 20" \
 "ct_base:200:$B python -u scripts/conv_micro.py --batch 384 --passes tdgrad,tdgradbn --only up --iters 20" \
 "b_base1:200:$B python -u bench.py --steps 20 --warmup 5" \
 "b_new1:200:python -u bench.py --steps 20 --warmup 5" \
 "b_base2:200:$B python -u bench.py --steps 20 --warmup 5" \
 "b_new2:200:python -u bench.py --steps 20 --warmup 5" \
 "b_base3:200:$B python -u bench.py --steps 20 --warmup 5" \
 "b_new3:200:python -u bench.py --steps 20 --warmup 5"
