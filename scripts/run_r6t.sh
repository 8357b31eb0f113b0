# transposed-conv forward with 256-wide column tiles (CONVT_FWD_BN256): numerics, per level, bench
scripts/gpu.sh r6t \
 "t:300:DDLPC_CONVT_FWD_BN256=1 python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'convt' --timeout 120 --timeout-method thread" \
 "ct:300:python -u scripts/conv_micro.py --batch 384 --passes tfwd,tfwdbn --only up --ab CONVT_FWD_BN256:0,1 --rounds 5 --iters 20" \
 "b:300:python -u bench.py --ab CONVT_FWD_BN256:0,1"
