set -e
O=gpurun_out/r01p; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_verify_gpu.py -m gpu -x -q -p no:cacheprovider > $O/pytest_verify.log 2>&1
timeout -k 10 300 python tools/tune_verify.py --variants 6,9,10,7 --bpc 8 --nt 1 --rounds 5 --launches 100 > $O/tune.json 2>&1
timeout -k 10 300 python tools/tune_verify.py --variants 6,9 --bpc 8 --nt 1 --rounds 5 --launches 100 --corrupt-rate 16 > $O/tune_c16.json 2>&1
