# BN-backward-epilogue data gradients on the BM-512 tiles (CONV_BNB_CFG5): numerics, per layer, bench
scripts/gpu.sh r6ag \
 "t:300:DDLPC_CONV_BNB_CFG5=1 python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'dgrad_bn_backward_epilogue' --timeout 120 --timeout-method thread" \
 "cm:400:python -u scripts/conv_micro.py --batch 384 --passes dgradbn --ab CONV_BNB_CFG5:0,1 --rounds 3 --iters 10" \
 "b:300:python -u bench.py --ab CONV_BNB_CFG5:0,1"
