# head kernels: slots refilled after their last use, branch-free steps (new) vs HEAD
D=distributed-deep-learning-on-personal-computers_amd/_lib/diag
B="DDLPC_LIB_PATH=$D/libddlpc_diag_head_ce_HEAD.so"
scripts/gpu.sh r6y \
 "t:300:python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'head' --timeout 120 --timeout-method thread" \
 "hm_base:120:$B python -u scripts/head_micro.py --batch 384 --iters 20" \
 "hm_new:120:python -u scripts/head_micro.py --batch 384 --iters 20" \
 "b_base1:200:$B python -u bench.py --steps 20 --warmup 5" \
 "b_new1:200:python -u bench.py --steps 20 --warmup 5" \
 "b_base2:200:$B python -u bench.py --steps 20 --warmup 5" \
 "b_new2:200:python -u bench.py --steps 20 --warmup 5"
