# Headline leg at the driver's settings vs longer warmup / more steps: where the 20-step penalty comes from.
set -e
O=gpurun_out/${1:-ov}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras > $O/w5_$r.json 2>> $O/err.log
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --warmup 50 > $O/w50_$r.json 2>> $O/err.log
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 200 > $O/s200_$r.json 2>> $O/err.log
done
