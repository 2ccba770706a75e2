set -euo pipefail
OUT=gpurun_out/r03h; mkdir -p $OUT
export TMPDIR=/tmp
echo "[$(date +%T)] tests" >> $OUT/steps.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_media_stream.py -m gpu -k "frames or udp_status or end_to_end" > $OUT/pytest.log 2>&1
echo "[$(date +%T)] probe" >> $OUT/steps.log
timeout -k 10 300 python tools/media_stream_probe.py --datagrams 16777216 --arenas 2 --only verify,verify_strided,ms+frames,ms_strided+frames,ms_strided+status_v3,ms+status --ms-variants 3 --launches 10 --rounds 3 > $OUT/ms_probe.jsonl 2> $OUT/ms_probe.err
echo "[$(date +%T)] done" >> $OUT/steps.log
