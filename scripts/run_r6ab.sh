# head forward: conflict-free (XOR-swizzled) dWh transposes vs HEAD
D=distributed-deep-learning-on-personal-computers_amd/_lib/diag
B="DDLPC_LIB_PATH=$D/libddlpc_diag_head_ce_HEAD.so"
scripts/gpu.sh r6ab \
 "t:300:python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'head' --timeout 120 --timeout-method thread" \
 "hm_base:120:$B python -u scripts/head_micro.py --batch 384 --iters 20" \
 "hm_new:120:python -u scripts/head_micro.py --batch 384 --iters 20" \
 "hm_base2:120:$B python -u scripts/head_micro.py --batch 384 --iters 20" \
 "hm_new2:120:python -u scripts/head_micro.py --batch 384 --iters 20" \
 "pmc:200:PMC='SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE' bash scripts/pmc_head.sh gpurun_out/r6ab/pmc --batch 384" \
 "b_base1:200:$B python -u bench.py --steps 20 --warmup 5" \
 "b_new1:200:python -u bench.py --steps 20 --warmup 5" \
 "b_base2:200:$B python -u bench.py --steps 20 --warmup 5" \
 "b_new2:200:python -u bench.py --steps 20 --warmup 5"
