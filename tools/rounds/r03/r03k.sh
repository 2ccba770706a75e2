set -euo pipefail
OUT=gpurun_out/r03k; mkdir -p $OUT
echo "[$(date +%T)] fill probe" >> $OUT/steps.log
timeout -k 10 300 python tools/media_stream_probe.py --datagrams 16777216 --arenas 2 --launches 5 --rounds 3 \
  --only fill_payload,ms_fill,verify_strided > $OUT/fill_probe.jsonl 2> $OUT/fill_probe.err
echo "[$(date +%T)] write ceiling" >> $OUT/steps.log
timeout -k 10 120 tools/write_shape_probe > $OUT/write_shape.jsonl 2> $OUT/write_shape.err || true
echo "[$(date +%T)] done" >> $OUT/steps.log
