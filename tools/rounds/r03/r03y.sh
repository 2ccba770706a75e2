set -euo pipefail
OUT=gpurun_out/r03y; mkdir -p $OUT
echo "[$(date +%T)] tests" >> $OUT/steps.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_media_stream.py tests/test_verify_gpu.py -m gpu -k "fill or end_to_end or materialize or config3" > $OUT/pytest.log 2>&1
echo "[$(date +%T)] ring probe" >> $OUT/steps.log
timeout -k 10 240 tools/ring_fill_probe 16777216 2 > $OUT/ring_fill.jsonl 2> $OUT/ring_fill.err
echo "[$(date +%T)] done" >> $OUT/steps.log
