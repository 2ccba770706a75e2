# round 3: MediaStream patterns of the ctsIoPattern mirror on the GPU, then the whole GPU suite and smoke
set -euo pipefail
OUT=gpurun_out/ms_pattern; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_media_stream_pattern.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_ms_pattern.log 2>&1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
