# round 3: roofline leg from host launches (--no-serial-graph) vs HIP-graph replays (the default), A/B on one box
set -euo pipefail
OUT=gpurun_out/serial_graph3; mkdir -p $OUT
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --no-engines-leg --no-serial-graph > $OUT/host_$r.json 2> $OUT/host_$r.err
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --no-engines-leg > $OUT/graph_$r.json 2> $OUT/graph_$r.err
done
timeout -k 10 300 python -u -m pytest tests/test_bench_engines.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
