set -euo pipefail
OUT=gpurun_out/r03j; mkdir -p $OUT
echo "[$(date +%T)] tests" >> $OUT/steps.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_media_stream.py tests/test_loopback.py -m gpu -k "frames or randomized" > $OUT/pytest.log 2>&1
echo "[$(date +%T)] bench" >> $OUT/steps.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
echo "[$(date +%T)] dist" >> $OUT/steps.log
bash tools/r03_dist8.sh r03j_dist
echo "[$(date +%T)] done" >> $OUT/steps.log
