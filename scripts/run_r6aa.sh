# head forward: two steps in lockstep (new: 4 WG/CU with a small spill, and 3 WG/CU) vs HEAD
D=distributed-deep-learning-on-personal-computers_amd/_lib/diag
B="DDLPC_LIB_PATH=$D/libddlpc_diag_head_ce_HEAD.so"
O3="DDLPC_LIB_PATH=$D/libddlpc_diag_head_ce_HEAD32_OCC3.so"
scripts/gpu.sh r6aa \
 "t:300:python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'head' --timeout 120 --timeout-method thread" \
 "t3:300:$O3 python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'head' --timeout 120 --timeout-method thread" \
 "hm_base:120:$B python -u scripts/head_micro.py --batch 384 --iters 20" \
 "hm_new:120:python -u scripts/head_micro.py --batch 384 --iters 20" \
 "hm_o3:120:$O3 python -u scripts/head_micro.py --batch 384 --iters 20" \
 "hm_base2:120:$B python -u scripts/head_micro.py --batch 384 --iters 20" \
 "hm_new2:120:python -u scripts/head_micro.py --batch 384 --iters 20" \
 "hm_o32:120:$O3 python -u scripts/head_micro.py --batch 384 --iters 20"
