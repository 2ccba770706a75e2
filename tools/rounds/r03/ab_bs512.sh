# tuning variant 21 (variant 13 at 512-thread workgroups) against the product shape (13), config-2 verify
set -euo pipefail
OUT=gpurun_out/ab_bs512; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_verify_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "test_launch_variants_parity and (21 or 13)" -p no:cacheprovider > $OUT/parity.log 2>&1
for r in 1 2; do
timeout -k 10 200 python tools/tune_verify.py --variants 13,21 --bpc 4,8,16 --nt 1 --rounds 5 --launches 40 --results > $OUT/tune_$r.json 2> $OUT/tune_$r.err
done
