scripts/gpu.sh r6j \
 "dec3:300:python -u scripts/conv_micro.py --batch 384 --only dec3.a --passes fwd,dgrad --ab CONV_DBG:0,1,2,4,8,3,9,12 --rounds 3" \
 "enc4:300:python -u scripts/conv_micro.py --batch 384 --only enc4.b --passes fwd,dgradbn --ab CONV_DBG:0,1,2,4,8,3,9,12 --rounds 3" \
 "dec4:300:python -u scripts/conv_micro.py --batch 384 --only dec4.a --passes fwd --ab CONV_DBG:0,1,2,4,8,3,9,12 --rounds 3"
