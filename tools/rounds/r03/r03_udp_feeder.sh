# round 3: MediaStream over loopback UDP with the GPU verify (per datagram and batched), and the MediaStream pattern tests
set -euo pipefail
OUT=gpurun_out/udp_feeder4; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_loopback_media_stream.py tests/test_media_stream_pattern.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
timeout -k 10 200 python -c "
import json, sys
sys.path.insert(0, '.')
from ctstraffic_amd import Engine, loopback as LB
with Engine(0) as e:
    for mode in (0, 1):
        for n in (1, 4, 16):
            r = LB.media_stream_run(connections=n, frame_size=52083, frames_per_second=240, stream_length_frames=240, buffered_frames=60, engine=e, verify_mode=mode)
            r['recv_cpu_us_per_datagram'] = 1e6 * r['recv_cpu_seconds'] / max(1, r['datagrams_received'])
            print(json.dumps({'verify_mode': ['SYNC', 'DEFERRED'][mode], 'connections': n, **r}), flush=True)
" > $OUT/runs.jsonl 2> $OUT/runs.err
