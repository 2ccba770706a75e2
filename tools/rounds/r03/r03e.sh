set -euo pipefail
OUT=gpurun_out/r03e; mkdir -p $OUT
sed -i 's/--rounds 3 --launches 10/--rounds 5 --launches 10/' tools/r03_dg_probe.sh
VARIANTS=9,13 NTS=1 bash tools/r03_dg_probe.sh r03e_dg
echo "[$(date +%T)] gpu tests" >> $OUT/steps.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_media_stream.py tests/test_io_pattern.py tests/test_loopback.py tests/test_status.py -m gpu > $OUT/pytest.log 2>&1
echo "[$(date +%T)] loopback bench" >> $OUT/steps.log
timeout -k 10 300 python bench.py --extras-only loopback --steps 5 --cpu-seconds 1 > $OUT/bench_loopback.json 2> $OUT/bench_loopback.err
timeout -k 10 300 python bench.py --extras-only loopback --steps 5 --no-cpu-baseline > $OUT/bench_loopback2.json 2> $OUT/bench_loopback2.err
echo "[$(date +%T)] done" >> $OUT/steps.log
