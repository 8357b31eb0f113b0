# GPU suite after the device-parametrised engine tests and the codec routing
scripts/gpu.sh r6ao \
 "tests:1000:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread"
