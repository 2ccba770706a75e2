set -euo pipefail
O=gpurun_out/r05b; mkdir -p $O; export TMPDIR=/tmp
echo "[$(date +%T)] pytest" 
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "[$(date +%T)] ab"
for i in 1 2 3; do
  timeout -k 10 90 tools/ab/verify_timeline_r04 2 64 > $O/tl_r04_$i.jsonl 2>&1
  timeout -k 10 90 tools/verify_timeline 2 64 > $O/tl_r05_$i.jsonl 2>&1
done
echo "[$(date +%T)] tail"
timeout -k 10 150 tools/verify_timeline 3 64 tail > $O/tail.jsonl 2>&1
echo "[$(date +%T)] bench"
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
echo "[$(date +%T)] engines"
timeout -k 10 240 python bench.py --engines 1 --no-cpu-baseline --no-extras > $O/engines1.json 2> $O/engines1.err
timeout -k 10 240 python bench.py --engines 2 --engines-same-gpu --no-cpu-baseline --no-extras > $O/engines2same.json 2> $O/engines2same.err
echo "[$(date +%T)] done"
