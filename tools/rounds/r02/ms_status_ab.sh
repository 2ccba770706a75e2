# Compact MediaStream receive (16-byte statuses) vs records + results: parity first, then an A/B at 16 M datagrams.
set -e
O=gpurun_out/${1:-msstatus}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_media_stream.py tests/test_abi.py tests/test_verify_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "media_stream or product_build or product_library" > $O/pytest.log 2>&1
timeout -k 10 300 python -u tools/media_stream_probe.py --datagrams 16777216 --arenas 2 --launches 10 --rounds 3 \
  --only ms,ms+records+results,ms+status,ms+status_every_round,ms+status_ring16,ms+status_ring32,ms_strided+status,verify > $O/probe_16M.jsonl 2> $O/probe.err
