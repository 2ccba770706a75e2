set -e
O=gpurun_out/r01q; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python tools/tune_verify.py --variants 6,9,10 --bpc 8 --nt 1 --rounds 9 --launches 100 > $O/tune.json 2>&1
timeout -k 10 300 python tools/tune_verify.py --variants 10,9 --bpc 9,12,16 --nt 1 --rounds 3 --launches 100 > $O/tune_bpc.json 2>&1
