set -e
O=gpurun_out/r01l; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python tools/tune_verify.py --variants 6,8,0 --bpc 8 --nt 1 --rounds 5 --launches 100 > $O/tune.json 2>&1
timeout -k 10 300 python tools/tune_verify.py --workload datagram --variants 0,3,4 --bpc 32,64 --nt 1 --rounds 3 --launches 10 > $O/tune_dgram.json 2>&1
