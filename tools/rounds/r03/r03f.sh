set -euo pipefail
OUT=gpurun_out/r03f; mkdir -p $OUT
sed -i 's/--rounds 3 --launches 10/--rounds 5 --launches 10/' tools/r03_dg_probe.sh
VARIANTS=9,13,15 NTS=1 bash tools/r03_dg_probe.sh r03f_dg
echo "[$(date +%T)] loopback probe" >> $OUT/steps.log
timeout -k 10 300 python tools/loopback_probe.py --cases deferred_sync_ab --rounds 3 > $OUT/loopback_probe.jsonl 2> $OUT/loopback_probe.err
echo "[$(date +%T)] io tests" >> $OUT/steps.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_io_pattern.py tests/test_loopback.py -m gpu > $OUT/pytest.log 2>&1
echo "[$(date +%T)] done" >> $OUT/steps.log
