set -euo pipefail
OUT=gpurun_out/r03o; mkdir -p $OUT
echo "[$(date +%T)] ring fill probe" >> $OUT/steps.log
timeout -k 10 240 tools/ring_fill_probe 16777216 2 > $OUT/ring_fill.jsonl 2> $OUT/ring_fill.err
echo "[$(date +%T)] tests" >> $OUT/steps.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_media_stream.py -m gpu -k "fill or end_to_end" > $OUT/pytest.log 2>&1
echo "[$(date +%T)] done" >> $OUT/steps.log
