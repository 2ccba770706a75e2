#!/bin/bash
# One gpurun call (round 6): the GPU suite (the DataError count and the prepared RCCL clique included), the rotated
# write-ceiling probe beside the product fill, the fill->verify pairs with their PMC passes, the engines legs and the
# default bench line. Every GPU step has its own time limit and the steps chain under set -e: after a failure nothing
# more runs on the GPU.
#   usage (from this container):  make all probes && gpurun --timeout 1100 -- bash tools/gpu_r06.sh TAG [STEPS]
set -euo pipefail
O=gpurun_out/${1:-r06}; mkdir -p "$O"; export TMPDIR=/tmp
STEPS=${2:-tests,ceiling,pairs,engines,bench}
run() { echo "[$(date +%T)] $*" | tee -a "$O/steps.log"; }
if [[ $STEPS == *tests* ]]; then
  run pytest-gpu
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > "$O/pytest_gpu.log" 2>&1
  run smoke
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
fi
if [[ $STEPS == *ceiling* ]]; then
  # SWEEP=0: slab vs grid-strided stores at 4/8/16 waves per CU; SWEEP=1: store width and the piece-order fill
  run write-ceiling-rotated
  SWEEP=${SWEEP:-1} timeout -k 10 240 tools/write_ceiling_rot > "$O/write_ceiling_rotated.jsonl" 2> "$O/write_ceiling_rotated.err"
fi
if [[ $STEPS == *pairs* ]]; then
  run fill-verify-pairs
  timeout -k 10 120 python tools/fill_verify_pairs.py > "$O/fill_verify_pairs.json" 2> "$O/fill_verify_pairs.err"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    run fill-verify-pairs-pmc $ctr
    timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d "$O/pairs_pmc_$ctr" -o run --output-format csv \
      -- python3 tools/fill_verify_pairs.py > "$O/pairs_pmc_$ctr.json" 2> "$O/pairs_pmc_$ctr.err"
  done
fi
if [[ $STEPS == *pairsprof* ]]; then
  # the fill+verify pairs under the kernel trace: per-launch durations of the rotated fill and verify
  run fill-verify-pairs-kernel-trace
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$O/pairs_kt" -o run --output-format csv \
    -- python3 tools/fill_verify_pairs.py > "$O/pairs_kt.json" 2> "$O/pairs_kt.err"
fi
if [[ $STEPS == *engines* ]]; then
  run engines
  timeout -k 10 300 python bench.py --engines 1 --no-cpu-baseline --no-extras > "$O/bench_engines1.json" 2> "$O/bench_engines1.err"
  timeout -k 10 300 python bench.py --engines 2 --engines-same-gpu --no-cpu-baseline --no-extras \
    > "$O/bench_engines2same.json" 2> "$O/bench_engines2same.err"
fi
if [[ $STEPS == *fillx* ]]; then
  # the fill extras alone (fill_GBps, the fill+verify pairs) through the C ABI
  run bench-fill-extras
  timeout -k 10 300 python bench.py --no-cpu-baseline --extras-only fill --no-engines-leg --steps 5 --warmup 2 \
    > "$O/bench_fill.json" 2> "$O/bench_fill.err"
fi
if [[ $STEPS == *dgx* ]]; then
  # the datagram extras alone (config-3 verify, MediaStream receive forms and fills)
  run bench-datagram-extras
  timeout -k 10 300 python bench.py --no-cpu-baseline --extras-only datagram --no-engines-leg --steps 5 --warmup 2 \
    > "$O/bench_datagram.json" 2> "$O/bench_datagram.err"
fi
if [[ $STEPS == *bench* ]]; then
  run bench
  timeout -k 10 500 python bench.py > "$O/bench.json" 2> "$O/bench.err"
fi
run done
