set -e
O=gpurun_out/r01n; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_verify_gpu.py -m gpu -x -q -p no:cacheprovider > $O/pytest_verify.log 2>&1
timeout -k 10 300 python tools/tune_verify.py --variants 6,9,10,1 --bpc 8 --nt 1 --rounds 5 --launches 100 > $O/tune.json 2>&1
timeout -k 10 300 python tools/tune_verify.py --variants 6,9,10 --bpc 4,12 --nt 1 --rounds 3 --launches 100 > $O/tune_bpc.json 2>&1
