set -e
mkdir -p gpurun_out/ov
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras > gpurun_out/ov/b$r.json 2>> gpurun_out/ov/err.log
done
timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 200 > gpurun_out/ov/b200.json 2>> gpurun_out/ov/err.log
