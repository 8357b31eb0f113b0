# 64-channel layers on 512-pixel 8-wave tiles (CONV_CFG10): numerics, per layer, bench
scripts/gpu.sh r6ai \
 "t:400:DDLPC_CONV_CFG10=1 python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'conv3_fwd or conv3_dgrad' --timeout 120 --timeout-method thread" \
 "cm:400:python -u scripts/conv_micro.py --batch 384 --passes fwd,dgrad,dgradbn --ab CONV_CFG10:0,1 --rounds 3 --iters 10" \
 "b:300:python -u bench.py --ab CONV_CFG10:0,1"
