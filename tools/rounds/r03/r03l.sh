set -euo pipefail
OUT=gpurun_out/r03l; mkdir -p $OUT
echo "[$(date +%T)] tests" >> $OUT/steps.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_media_stream.py tests/test_verify_gpu.py -m gpu -k "fill or end_to_end" > $OUT/pytest.log 2>&1
echo "[$(date +%T)] fill probe" >> $OUT/steps.log
timeout -k 10 300 python tools/media_stream_probe.py --datagrams 16777216 --arenas 2 --launches 5 --rounds 3 \
  --only fill_payload,fill_payload_plain,ms_fill,ms_fill_plain,verify_strided > $OUT/fill_probe.jsonl 2> $OUT/fill_probe.err
echo "[$(date +%T)] done" >> $OUT/steps.log
