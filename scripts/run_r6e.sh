scripts/gpu.sh r6e \
 "tk:300:python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k 'convt'" \
 "tdata:300:python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_data_gpu.py -k prefetcher" \
 "abfb8:400:python -u bench.py --steps 10 --warmup 5 --ab CONVT_FB8:0,1 --ab-rounds 4" \
 "base384:900:python -u bench.py --impl torch --batch 384 --steps 10 --warmup 3 --heartbeat 20 --verbose 1"
