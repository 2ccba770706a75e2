set -euo pipefail
OUT=gpurun_out/r03r; mkdir -p $OUT
timeout -k 10 240 tools/ring_fill_probe 16777216 2 > $OUT/ring_fill.jsonl 2> $OUT/ring_fill.err
