# head forward: branch-free steps with per-step LDS scratch (new, 4 WG/CU) vs the HEAD kernel vs 3 WG/CU
D=distributed-deep-learning-on-personal-computers_amd/_lib/diag
B="DDLPC_LIB_PATH=$D/libddlpc_diag_head_ce_HEAD.so"
O3="DDLPC_LIB_PATH=$D/libddlpc_diag_head_ce_HEAD32_OCC3.so"
scripts/gpu.sh r6q \
 "t:300:python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'head' --timeout 120 --timeout-method thread" \
 "t3:300:$O3 python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'head' --timeout 120 --timeout-method thread" \
 "hm_base:120:$B python -u scripts/head_micro.py --batch 384 --iters 20" \
 "hm_new:120:python -u scripts/head_micro.py --batch 384 --iters 20" \
 "hm_o3:120:$O3 python -u scripts/head_micro.py --batch 384 --iters 20" \
 "b_base1:200:$B python -u bench.py --steps 20 --warmup 5" \
 "b_new1:200:python -u bench.py --steps 20 --warmup 5" \
 "b_o31:200:$O3 python -u bench.py --steps 20 --warmup 5" \
 "b_base2:200:$B python -u bench.py --steps 20 --warmup 5" \
 "b_new2:200:python -u bench.py --steps 20 --warmup 5" \
 "b_o32:200:$O3 python -u bench.py --steps 20 --warmup 5"
