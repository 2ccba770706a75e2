# receive-thread CPU inside the pattern calls (tools/pattern_cpu_probe), 1 and 8 connections at once
set -e
mkdir -p gpurun_out/pcp
for r in 1 2; do
  for m in "off 1 0" "sync 1 0" "deferred 1 1024" "deferred 1 4096"; do
    timeout -k 10 60 tools/pattern_cpu_probe $m 1 >> gpurun_out/pcp/probe.jsonl
    timeout -k 10 60 tools/pattern_cpu_probe $m 8 >> gpurun_out/pcp/probe.jsonl
  done
  CTS_DEFERRED_BLOCKING_SYNC=0 timeout -k 10 60 tools/pattern_cpu_probe deferred 1 1024 8 >> gpurun_out/pcp/probe.jsonl
done
