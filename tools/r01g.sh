set -e
O=gpurun_out/r01g; mkdir -p $O; export TMPDIR=/tmp
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
for set in "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -k 10 200 rocprofv3 --pmc $set --kernel-trace -T -d $O/pmc_$tag -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras --steps 30 --warmup 5 > $O/pmc_$tag.bench.json 2> $O/pmc_$tag.err
  timeout -k 10 200 rocprofv3 --pmc $set --kernel-trace -T -d $O/abl_$tag -o run --output-format csv -- ./tools/verify_ablation 20 > $O/abl_$tag.jsonl 2> $O/abl_$tag.err
done
