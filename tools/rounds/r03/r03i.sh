set -euo pipefail
OUT=gpurun_out/r03i; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_media_stream.py -m gpu -k "frames" > $OUT/pytest.log 2>&1
bash tools/r03_dist8.sh r03_dist8
