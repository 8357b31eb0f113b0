# in-house MIOpen baseline at per-GPU batch 384 (first step runs MIOpen's find for every conv shape)
mkdir -p gpurun_out/r6f
export TMPDIR=/tmp
timeout -k 10 1150 python -u bench.py --impl torch --batch 384 --steps 10 --warmup 2 --heartbeat 20 --verbose 1 > gpurun_out/r6f/base384.log 2>&1
