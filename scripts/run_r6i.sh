scripts/gpu.sh r6i \
 "pf1:200:python -u bench.py --steps 20 --warmup 5" \
 "pf0:200:python -u bench.py --steps 20 --warmup 5 --prefetch 0" \
 "pf1b:200:python -u bench.py --steps 20 --warmup 5" \
 "pf0b:200:python -u bench.py --steps 20 --warmup 5 --prefetch 0" \
 "proxy:300:python -u bench.py --steps 10 --warmup 5 --comm-proxy 8" \
 "trace:400:rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6i/tr -o run -- python3 bench.py --steps 4 --warmup 3 --schedule serial" \
 "sum:60:f=\$(find gpurun_out/r6i/tr -name '*kernel_trace.csv' | head -1); python scripts/trace_summary.py \$f 4 list > gpurun_out/r6i/serial_list.txt; rm -rf gpurun_out/r6i/tr"
