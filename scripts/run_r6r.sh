# deferred encoder skips (pre-BN skip, BN + ReLU on load in the decoder) by level, same box
scripts/gpu.sh r6r \
 "b_off1:200:python -u bench.py --steps 20 --warmup 5" \
 "b_l0a:200:python -u bench.py --steps 20 --warmup 5 --engine-set defer_skip=1,defer_skip_max_level=0" \
 "b_l1a:200:python -u bench.py --steps 20 --warmup 5 --engine-set defer_skip=1,defer_skip_max_level=1" \
 "b_alla:200:python -u bench.py --steps 20 --warmup 5 --engine-set defer_skip=1" \
 "b_off2:200:python -u bench.py --steps 20 --warmup 5" \
 "b_l0b:200:python -u bench.py --steps 20 --warmup 5 --engine-set defer_skip=1,defer_skip_max_level=0" \
 "b_l1b:200:python -u bench.py --steps 20 --warmup 5 --engine-set defer_skip=1,defer_skip_max_level=1" \
 "b_allb:200:python -u bench.py --steps 20 --warmup 5 --engine-set defer_skip=1" \
 "prof_l0:300:rocprofv3 --kernel-trace --stats -d gpurun_out/r6r/prof_l0 -o run -- python3 bench.py --steps 3 --warmup 2 --schedule serial --engine-set defer_skip=1,defer_skip_max_level=0"
