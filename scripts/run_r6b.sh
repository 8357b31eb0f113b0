scripts/gpu.sh r6b \
 "b256a:200:python -u bench.py --steps 20 --warmup 5" \
 "b512a:200:python -u bench.py --steps 10 --warmup 3 --batch 512" \
 "b384a:200:python -u bench.py --steps 14 --warmup 4 --batch 384" \
 "b256b:200:python -u bench.py --steps 20 --warmup 5" \
 "b512b:200:python -u bench.py --steps 10 --warmup 3 --batch 512" \
 "abprio:400:python -u bench.py --steps 10 --warmup 5 --ab CONV_PRIO:0,1,2 --ab-rounds 3" \
 "t:300:python -u -m pytest -v --timeout 200 --timeout-method thread -s tests/test_unet_gpu.py -k 'flagship_gradients_tight or (window_matches_sequential and 64-6-2-2)'"
