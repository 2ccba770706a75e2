# MediaStream receive with records + results: written every round (tuning variant 11) vs from a per-wave LDS ring
# every 32 / 64 rounds (tuning variant 6 / variant 3, the product); parity first.
set -e
O=gpurun_out/${1:-msrec}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_media_stream.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "media_stream" > $O/pytest.log 2>&1
timeout -k 10 300 python -u tools/media_stream_probe.py --datagrams 16777216 --arenas 2 --launches 10 --rounds 3 \
  --ms-variants 3,11 --only ms,ms+records+results,ms_strided+records+results,ms+status,ms_strided+status > $O/probe_16M.jsonl 2> $O/probe.err
