set -e
O=gpurun_out/r01k; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1
timeout -k 10 200 ./tools/verify_ablation 200 > $O/ablation.jsonl 2>&1
timeout -k 10 600 python bench.py > $O/bench.json 2>&1
