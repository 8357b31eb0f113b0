scripts/gpu.sh r6d \
 "abxd:400:python -u bench.py --steps 10 --warmup 5 --ab CFG5_XD:4,6 --ab-rounds 4" \
 "base384:400:python -u bench.py --impl torch --batch 384 --steps 10 --warmup 3"
