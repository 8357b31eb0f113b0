scripts/gpu.sh r6b \
 "t:300:python -u -m pytest -x -v --timeout 200 --timeout-method thread -s tests/test_unet_gpu.py -k 'flagship_gradients_tight or (window_matches_sequential and 64-6-2-2)'"
