#!/bin/bash
# SYNC mailbox: one slot read in flight per poller (the round-2 grid) vs two, half a round trip apart
# (CTS_MAILBOX_POLLS), alternating, tools/sync_probe at 1 / 8 / 16 callers; then the mailbox GPU tests with two.
#   usage (from this container):  gpurun --timeout 900 -- bash tools/r03_polls_ab.sh TAG
set -euo pipefail
TAG=${1:-r03_polls}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in 1 2 3; do
  for p in 1 2; do
    echo "[$(date +%T)] round $r polls $p" >> "$OUT/steps.log"
    CTS_MAILBOX_POLLS=$p timeout -k 10 120 tools/sync_probe 2000 mailbox | sed "s/^{/{\"round\": $r, \"polls\": $p, /" >> "$OUT/sync_probe.jsonl"
  done
done
echo "[$(date +%T)] tests polls 2" >> "$OUT/steps.log"
CTS_MAILBOX_POLLS=2 timeout -k 10 300 python -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_verify_gpu.py -k "mailbox or host_free or verify_host or mapped" > "$OUT/pytest_polls2.log" 2>&1
echo "[$(date +%T)] done" >> "$OUT/steps.log"
