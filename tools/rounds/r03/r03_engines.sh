# round 3: the single-process leg with native launch threads (tools/bench_multi.cpp)
set -euo pipefail
OUT=gpurun_out/engines_native; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_bench_engines.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
timeout -k 10 200 python bench.py --engines 1 --no-cpu-baseline --no-extras > $OUT/engines1.json 2> $OUT/engines1.err
timeout -k 10 200 python bench.py --engines 4 --engines-same-gpu --no-cpu-baseline --no-extras > $OUT/engines4_same.json 2> $OUT/engines4_same.err
timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras > $OUT/bench_default.json 2> $OUT/bench_default.err
