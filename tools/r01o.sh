set -e
O=gpurun_out/r01o; mkdir -p $O; export TMPDIR=/tmp
for mb in 128 256 512 1024 2048; do
  echo "== $mb MiB" >> $O/ceiling_sizes.jsonl
  timeout -k 10 120 ./tools/hbm_read_ceiling 50 $mb 1 >> $O/ceiling_sizes.jsonl 2>&1
done
for nb in 2048 4096 8192 16384 32768; do
  echo "== $nb buffers" >> $O/verify_sizes.txt
  timeout -k 10 200 python tools/tune_verify.py --variants 6 --bpc 8 --nt 1 --rounds 3 --launches 50 --buffers $nb >> $O/verify_sizes.txt 2>&1
done
