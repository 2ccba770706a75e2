set -e
O=gpurun_out/r01r; mkdir -p $O; export TMPDIR=/tmp
PL=$PWD/ctstraffic_amd/build/pl/libcts_engine.so
CTS_ENGINE_LIB=$PL timeout -k 10 400 python -m pytest tests/test_verify_gpu.py -m gpu -x -q -p no:cacheprovider > $O/pytest_verify_pl.log 2>&1
for k in 1 2 3; do
  timeout -k 10 200 python tools/tune_verify.py --variants 10,6 --bpc 8,16 --nt 1 --rounds 3 --launches 100 > $O/tune_base_$k.json 2>&1
  CTS_ENGINE_LIB=$PL timeout -k 10 200 python tools/tune_verify.py --variants 10,6 --bpc 8,16 --nt 1 --rounds 3 --launches 100 > $O/tune_pl_$k.json 2>&1
done
