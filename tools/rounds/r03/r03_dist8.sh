#!/bin/bash
# Multi-rank rehearsal of the driver's SCALE command on the one-GPU box: bench.py --gpus N starts N ranks itself
# (gloo: nccl needs one GPU per rank), all on cuda:0, no extras; N = 4 and 8.
set -euo pipefail
OUT=gpurun_out/${1:-r03_dist8}
mkdir -p "$OUT"
for n in 4 8; do
  echo "[$(date +%T)] gpus $n" >> "$OUT/steps.log"
  timeout -k 10 400 python bench.py --gpus $n --dist-backend gloo --no-extras --cpu-seconds 2 --steps 20 --warmup 5 \
    > "$OUT/dist${n}_gloo.json" 2> "$OUT/dist${n}_gloo.err"
done
echo "[$(date +%T)] done" >> "$OUT/steps.log"
