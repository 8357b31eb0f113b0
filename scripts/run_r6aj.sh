# synthetic renderer: 32-bit shift geometry (new) vs HEAD
D=distributed-deep-learning-on-personal-computers_amd/_lib/diag
B="DDLPC_LIB_PATH=$D/libddlpc_diag_data_HEAD.so"
scripts/gpu.sh r6aj \
 \
 "s_base:120:$B python -u scripts/synth_micro.py" \
 "s_new:120:python -u scripts/synth_micro.py" \
 "b_base1:200:$B python -u bench.py --steps 20 --warmup 5" \
 "b_new1:200:python -u bench.py --steps 20 --warmup 5" \
 "b_base2:200:$B python -u bench.py --steps 20 --warmup 5" \
 "b_new2:200:python -u bench.py --steps 20 --warmup 5"
