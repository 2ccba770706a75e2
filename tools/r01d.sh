set -e
O=gpurun_out/r01d; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/tune_verify.py --variants 0,6,7,4 --bpc 8,16 --nt 1 --rounds 5 --launches 40 > $O/tune40.json 2>&1
timeout -k 10 300 python tools/tune_verify.py --variants 0,6,7 --bpc 8 --nt 1 --rounds 3 --launches 400 > $O/tune400.json 2>&1
timeout -k 10 120 ./tools/hbm_read_ceiling 400 > $O/ceiling400.jsonl 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/prof_kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras --steps 400 > $O/prof_bench.json 2> $O/prof.err
