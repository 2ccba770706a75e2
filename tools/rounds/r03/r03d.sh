set -euo pipefail
OUT=gpurun_out/r03d; mkdir -p $OUT
VARIANTS=9,13,14 NTS=1 bash tools/r03_dg_probe.sh r03d_dg
echo "[$(date +%T)] gpu tests" >> $OUT/steps.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_verify_gpu.py -k "mailbox or host_free" tests/test_media_stream.py tests/test_io_pattern.py tests/test_loopback.py > $OUT/pytest.log 2>&1
echo "[$(date +%T)] loopback bench" >> $OUT/steps.log
timeout -k 10 300 python bench.py --extras-only loopback --no-cpu-baseline --steps 5 > $OUT/bench_loopback.json 2> $OUT/bench_loopback.err
echo "[$(date +%T)] done" >> $OUT/steps.log
