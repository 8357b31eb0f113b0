# late epilogue stores (CONV_EPI_LATE): numerics with the knob on, per-layer A/B, bench A/B
scripts/gpu.sh r6p \
 "t:400:DDLPC_CONV_EPI_LATE=1 python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'conv3_fwd or conv3_dgrad or bn_group_fusion or conv3d_fwd' --timeout 120 --timeout-method thread" \
 "cm:500:python -u scripts/conv_micro.py --batch 384 --passes fwd,dgrad,dgradbn --ab CONV_EPI_LATE:0,1 --rounds 3" \
 "b:400:python -u bench.py --ab CONV_EPI_LATE:0,1"
