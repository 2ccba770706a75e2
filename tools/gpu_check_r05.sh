#!/bin/bash
# One gpurun call (round 5, late): the whole GPU suite on another box, and the verify beside a plain read of its own
# shape (tools/verify_timeline, product kernels) with this box's read ceiling.
#   usage (from this container):  gpurun --timeout 900 -- bash tools/gpu_check_r05.sh TAG
set -euo pipefail
O=gpurun_out/${1:-r05l}; mkdir -p "$O"; export TMPDIR=/tmp
echo "[$(date +%T)] pytest" | tee -a "$O/steps.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > "$O/pytest_gpu.log" 2>&1
for i in 1 2; do
  echo "[$(date +%T)] timeline $i" | tee -a "$O/steps.log"
  timeout -k 10 120 tools/verify_timeline 2 64 >> "$O/verify_timeline.jsonl" 2>> "$O/verify_timeline.err"
done
echo "[$(date +%T)] ceiling" | tee -a "$O/steps.log"
timeout -k 10 120 tools/hbm_read_ceiling 64 256 1 1 > "$O/ceiling.jsonl" 2> "$O/ceiling.err"
echo "[$(date +%T)] done" | tee -a "$O/steps.log"
