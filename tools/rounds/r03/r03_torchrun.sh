#!/bin/bash
# The driver's launch form: torch.distributed.run starts the ranks and bench.py sees WORLD_SIZE.
# N=1 with the default backend (RCCL), and N=2 over gloo with both ranks on this one GPU (a rehearsal:
# RCCL refuses two ranks on one GPU).
set -euo pipefail
OUT=gpurun_out/r03_torchrun
mkdir -p "$OUT"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/torchrun_n1.json" 2> "$OUT/torchrun_n1.err"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29512 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --no-extras --cpu-seconds 2 \
  > "$OUT/torchrun_n2_gloo.json" 2> "$OUT/torchrun_n2_gloo.err"
echo done
