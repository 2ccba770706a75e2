#!/bin/bash
# The config-2 verify of round 6 (kCounterCount 6: the DataError slot) against round 5's, alternated on one box, each
# beside a plain read of its shape (tools/verify_timeline.hip, verify_timeline_r05). Diagnostic, profiles/r06/h/.
set -euo pipefail
O=gpurun_out/${1:-r06w}; mkdir -p "$O"; export TMPDIR=/tmp
for rep in 1 2 3; do
  for t in verify_timeline verify_timeline_r05; do
    echo "[$(date +%T)] $t $rep" | tee -a "$O/steps.log"
    timeout -k 10 120 tools/$t 2 64 >> "$O/$t.jsonl" 2>> "$O/$t.err"
  done
done
