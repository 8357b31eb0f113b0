# BM-512 decomposition, part 2: fragment reads vs MFMA vs DMA (diagnostic libraries)
D=distributed-deep-learning-on-personal-computers_amd/_lib/diag
steps=()
for m in 0 1 2 3 6 7; do
  if [ $m = 0 ]; then L=""; else L="DDLPC_LIB_PATH=$D/libddlpc_diag_$m.so"; fi
  steps+=("m$m:240:$L python -u scripts/conv_micro.py --batch 384 --only dec3.a --passes fwd,dgrad --iters 20 && $L python -u scripts/conv_micro.py --batch 384 --only enc4.b --passes fwd --iters 20")
done
scripts/gpu.sh r6l "${steps[@]}"
