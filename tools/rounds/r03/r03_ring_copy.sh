# the recv copy's CPU into DEFERRED's pinned recv-ring slots vs the one hot buffer (tools/pattern_cpu_probe)
set -e
mkdir -p gpurun_out/rc
for r in 1 2; do
  for m in "off 1 0" "deferred 1 64" "deferred 1 1024" "deferred 1 4096"; do
    timeout -k 10 60 tools/pattern_cpu_probe $m 1 >> gpurun_out/rc/probe.jsonl
    timeout -k 10 60 tools/pattern_cpu_probe $m 8 >> gpurun_out/rc/probe.jsonl
  done
done
