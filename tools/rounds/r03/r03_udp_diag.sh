# diagnosis: DEFERRED MediaStream client on the GPU missing a corrupt datagram
set -uo pipefail
OUT=gpurun_out/udp_diag; mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_media_stream_pattern.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_pattern.log 2>&1
timeout -k 10 120 python -c "
import json, sys
sys.path.insert(0, '.')
from ctstraffic_amd import Engine, loopback as LB
with Engine(0) as e:
    for mode in (1, 0, 1):
        for ci in (20, 100, 1000):
            r = LB.media_stream_run(connections=1, frame_size=52083, frames_per_second=120, stream_length_frames=60, buffered_frames=30, engine=e, verify_mode=mode, corrupt_connection=0, corrupt_datagram=ci)
            print(json.dumps({'mode': mode, 'ci': ci, 'ok': r['connections_ok'], 'derr': r['data_errors'], 'frames': r['clients']['successful_frames']}), flush=True)
" > $OUT/diag.jsonl 2> $OUT/diag.err
