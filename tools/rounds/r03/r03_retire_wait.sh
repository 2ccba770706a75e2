# DEFERRED retire wait: blocking-sync event (1) vs sleep-poll (2, default), pattern-only probe and config-1 loopback
set -e
mkdir -p gpurun_out/rw
for r in 1 2 3; do
  for w in 1 2; do
    CTS_DEFERRED_BLOCKING_SYNC=$w timeout -k 10 60 tools/pattern_cpu_probe deferred 1 1024 8 | sed "s/^{/{\"wait\": $w, /" >> gpurun_out/rw/probe.jsonl
  done
done
timeout -k 10 300 python -u tools/loopback_probe.py --cases deferred_sync_ab --rounds 3 > gpurun_out/rw/loopback.jsonl
