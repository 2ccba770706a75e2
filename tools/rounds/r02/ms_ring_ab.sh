# A/B of output write frequency: MediaStream receive with a per-wave output ring (ms variants 4-6 vs 3)
# and the config-2 verify writing its result records 16 at a time (verify variant 18 vs 13); parity first.
set -e
O=gpurun_out/${1:-msring}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_media_stream.py tests/test_verify_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "matches_oracle or launch_variants_parity or staged_results or max_length" \
  > $O/pytest.log 2>&1
timeout -k 10 300 python -u tools/media_stream_probe.py --datagrams 16777216 --arenas 2 --launches 10 --rounds 3 \
  --ms-variants 3,4,5,6 --only ms,ms+records+results > $O/probe_16M.jsonl 2> $O/probe.err
for r in 1 2 3; do
  for v in 13 18; do
    timeout -k 10 120 python bench.py --verify-variant $v --no-cpu-baseline --no-extras > $O/bench_v${v}_$r.json 2>> $O/bench.err
  done
done
