#!/bin/bash
# MediaStream fills (descriptors / ring) at 1, 2, 4 and 8 workgroups per CU (CTS_RING_FILL_BLOCKS_PER_CU), alternated
# twice: the datagram extras of bench.py, one process per setting (diagnostic, profiles/r06/d/).
set -euo pipefail
O=gpurun_out/${1:-r06n}; mkdir -p "$O"; export TMPDIR=/tmp
for rep in 1 2; do
  for b in 1 2 4 8; do
    echo "[$(date +%T)] rep $rep blocks_per_cu $b" | tee -a "$O/steps.log"
    CTS_RING_FILL_BLOCKS_PER_CU=$b timeout -k 10 200 python bench.py --no-cpu-baseline --extras-only datagram \
      --no-engines-leg --steps 2 --warmup 1 > "$O/dg_b${b}_r${rep}.json" 2> "$O/dg_b${b}_r${rep}.err"
  done
done
