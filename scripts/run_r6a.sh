scripts/gpu.sh r6a bench \
 "trace:400:rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6a/tr -o run -- python3 bench.py --steps 4 --warmup 3 --schedule serial" \
 "sum:60:f=\$(find gpurun_out/r6a/tr -name '*kernel_trace.csv' | head -1); python scripts/trace_summary.py \$f 4 list > gpurun_out/r6a/serial_list.txt; rm -rf gpurun_out/r6a/tr"
