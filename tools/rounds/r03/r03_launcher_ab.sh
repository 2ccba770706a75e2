# round 3: headline leg with the launches issued from native code vs one ctypes call per launch (A/B, same box)
set -euo pipefail
OUT=gpurun_out/launcher_ab; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_bench_engines.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
for r in 1 2 3; do
  for l in python native; do
    timeout -k 10 200 python bench.py --launcher $l --no-cpu-baseline --no-extras --no-engines-leg > $OUT/${l}_$r.json 2> $OUT/${l}_$r.err
  done
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --launcher native --pipeline-streams 1 > $OUT/native_s1.json 2> $OUT/native_s1.err
timeout -k 10 300 python bench.py --no-cpu-baseline --extras-only shards > $OUT/default_engines.json 2> $OUT/default_engines.err
