set -e
O=gpurun_out/r01s; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python tools/tune_verify.py --variants 10,9 --bpc 8,16,24,32,64 --nt 1 --rounds 7 --launches 100 > $O/tune_bpc.json 2>&1
timeout -k 10 300 python tools/tune_verify.py --variants 10,6 --bpc 8,16 --nt 1 --rounds 7 --launches 100 > $O/tune_b.json 2>&1
