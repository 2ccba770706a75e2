set -e
O=gpurun_out/r01j; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras > $O/bench_new_$i.json 2>&1
timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --stream default > $O/bench_default_$i.json 2>&1
timeout -k 10 120 python bench.py --no-cpu-baseline --no-extras --steps 100 --warmup 100 > $O/bench_k100_$i.json 2>&1
done
timeout -k 10 300 python tools/tune_verify.py --variants 0,6 --bpc 8 --nt 1 --rounds 3 --launches 200 > $O/tune_l200.json 2>&1
