set -euo pipefail
OUT=gpurun_out/r03g; mkdir -p $OUT
export TMPDIR=/tmp
P="tools/media_stream_probe.py --datagrams 16777216 --arenas 2 --ms-variants 3,12 --small-variants 9,15 --only verify,ms+records+results,verify_strided,ms_strided+status_v3,ms_strided+status_v12"
echo "[$(date +%T)] tests" >> $OUT/steps.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_media_stream.py tests/test_verify_gpu.py -m gpu -k "media_stream or small_variants or product_build or max_length or config3 or strided" > $OUT/pytest.log 2>&1
echo "[$(date +%T)] probe" >> $OUT/steps.log
timeout -k 10 300 python $P --launches 10 --rounds 3 > $OUT/ms_probe.jsonl 2> $OUT/ms_probe.err
echo "[$(date +%T)] pmc" >> $OUT/steps.log
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python3 $P --launches 2 --rounds 1 > $OUT/pmc_fetch.jsonl 2> $OUT/pmc_fetch.err
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python3 $P --launches 2 --rounds 1 > $OUT/pmc_write.jsonl 2> $OUT/pmc_write.err
echo "[$(date +%T)] done" >> $OUT/steps.log
