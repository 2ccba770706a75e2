#!/bin/bash
# Round 3: where the config-3 datagram verify's extra HBM reads come from (VERDICT r02 "Next round" 2).
# Small variants 9 (product) and 10-12 (line policies of quad_scan_interior), nt on/off, timed in one
# process (tools/tune_verify.py, 4 M datagrams, 2 rotated arenas), then the same command under PMC passes.
#   usage (from this container):  gpurun --timeout 1100 -- bash tools/r03_dg_probe.sh TAG
set -euo pipefail
TAG=${1:-r03b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { echo "[$(date +%T)] $*" | tee -a "$OUT/steps.log"; }
TV="tools/tune_verify.py --workload config3 --variants ${VARIANTS:-9,10,11,12} --bpc 64 --nt ${NTS:-1,0} --arenas 2"
run counters
timeout -k 10 60 rocprofv3 --list-avail > "$OUT/counters.txt" 2>&1 || true
run parity
timeout -k 10 300 python -m pytest tests/test_verify_gpu.py -x -q -p no:cacheprovider -k "small_variants_parity" > "$OUT/parity.log" 2>&1
run timing
timeout -k 10 300 python tools/tune_verify.py --workload config3 --variants ${VARIANTS:-9,10,11,12} --bpc 64 --nt ${NTS:-1,0} --arenas 2 --rounds 3 --launches 10 > "$OUT/timing.json" 2> "$OUT/timing.err"
for ctr in FETCH_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  tag=$(echo $ctr | tr ' ' '+')
  run pmc $tag
  timeout -k 10 240 rocprofv3 --pmc $ctr --kernel-trace -d "$OUT/pmc_$tag" -o run --output-format csv \
    -- python3 $TV --rounds 1 --launches 3 > "$OUT/pmc_$tag.json" 2> "$OUT/pmc_$tag.err"
done
run done
