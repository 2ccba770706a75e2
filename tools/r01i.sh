set -e
O=gpurun_out/r01i; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python tools/tune_verify.py --variants 0,6,3 --bpc 8 --nt 1 --rounds 5 --launches 100 --corrupt-rate 0 > $O/tune_c0.json 2>&1
timeout -k 10 300 python tools/tune_verify.py --variants 0,6,3 --bpc 8 --nt 1 --rounds 5 --launches 100 --corrupt-rate 1024 > $O/tune_c1024.json 2>&1
timeout -k 10 300 python tools/tune_verify.py --variants 0,6 --bpc 8 --nt 1 --rounds 3 --launches 100 --corrupt-rate 16 > $O/tune_c16.json 2>&1
timeout -k 10 600 python bench.py > $O/bench.json 2>&1
