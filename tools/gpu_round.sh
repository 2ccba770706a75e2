#!/bin/bash
# One gpurun call: GPU parity tests, smoke, bench, rocprofv3 kernel-trace stats and
# PMC HBM-traffic passes. Every GPU step has its own time limit; steps chain with &&
# semantics (set -e), so nothing more runs on the GPU after a failure.
#   usage (from this container):  make probes && gpurun --timeout 1100 -- bash tools/gpu_round.sh TAG
#   (the ceiling / timeline steps run the probes of `make probes`)
set -euo pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-all}
run() { echo "[$(date +%T)] $*" | tee -a "$OUT/steps.log"; }
if [[ $STEPS == all || $STEPS == *tests* ]]; then
  run pytest-gpu
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
  run smoke
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
fi
if [[ $STEPS == all || $STEPS == *bench* ]]; then
  run bench
  timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
fi
if [[ $STEPS == all || $STEPS == *engines* ]]; then
  # single-process multi-GPU leg (the ctsTraffic process model) at the GPUs this box has
  run engines
  timeout -k 10 300 python bench.py --engines 1 --no-cpu-baseline --no-extras > "$OUT/bench_engines1.json" 2> "$OUT/bench_engines1.err"
  # two engines sharing this GPU: the node-wide fold and RCCL all-reduce over two blocks (one device, one rank)
  timeout -k 10 300 python bench.py --engines 2 --engines-same-gpu --no-cpu-baseline --no-extras \
    > "$OUT/bench_engines2same.json" 2> "$OUT/bench_engines2same.err"
fi
if [[ $STEPS == all || $STEPS == *ceiling* ]]; then
  # plain streaming-read reference on the same box (build: see tools/hbm_read_ceiling.hip)
  run ceiling
  timeout -k 10 120 tools/hbm_read_ceiling 64 256 1 1 > "$OUT/ceiling.jsonl" 2> "$OUT/ceiling.err"
fi
if [[ $STEPS == all || $STEPS == *dist* ]]; then
  # 2-rank rehearsal of the multi-GPU path on this one GPU (gloo; both ranks on cuda:0)
  run dist-rehearsal
  # bench.py --gpus 2 starts its two ranks itself (a child torch.distributed.run), both on this one GPU over gloo
  timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --no-extras --cpu-seconds 2 --steps 50 --warmup 5 \
    > "$OUT/dist2_gloo.json" 2> "$OUT/dist2_gloo.err"
fi
if [[ $STEPS == all || $STEPS == *prof* ]]; then
  run rocprof-kernel-trace
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_kt" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-extras --pipeline-streams 1 --steps 200 --warmup 20 > "$OUT/prof_kt_bench.json" 2> "$OUT/prof_kt.err"
  for ctr in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum; do
    run rocprof-pmc $ctr
    timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace -T -d "$OUT/prof_pmc_$ctr" -o run --output-format csv \
      -- python3 bench.py --no-cpu-baseline --no-extras --pipeline-streams 1 --steps 50 --warmup 5 > "$OUT/prof_pmc_$ctr.json" 2> "$OUT/prof_pmc_$ctr.err"
  done
  # the default (pipelined) headline command under the kernel trace: its serialized roofline leg and
  # its pipelined leg as two bursts (tools/prof_summary.py: wall per launch, overlap)
  run rocprof-pipelined-kernel-trace
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_pipe_kt" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-extras --steps 200 --warmup 20 > "$OUT/prof_pipe_kt_bench.json" 2> "$OUT/prof_pipe_kt.err"
fi
if [[ $STEPS == all || $STEPS == *dgprof* ]]; then
  # config 3 (16 M datagrams): the bench's datagram extras under the same two profilers
  run rocprof-datagram-kernel-trace
  # (no -T: the MediaStream kernel's descriptor and strided-ring forms differ only in a template argument)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_dg_kt" -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --extras-only datagram --steps 5 --warmup 2 > "$OUT/prof_dg_kt_bench.json" 2> "$OUT/prof_dg_kt.err"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    run rocprof-datagram-pmc $ctr
    timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace -d "$OUT/prof_dg_pmc_$ctr" -o run --output-format csv \
      -- python3 bench.py --no-cpu-baseline --extras-only datagram --steps 5 --warmup 2 > "$OUT/prof_dg_pmc_$ctr.json" 2> "$OUT/prof_dg_pmc_$ctr.err"
  done
fi
if [[ $STEPS == *timeline* ]]; then
  # the product verify kernel beside a plain read of the same shape: times and per-workgroup timelines,
  # without and with the kernel arguments preloaded into SGPRs (tools/verify_timeline.hip)
  for rep in 1 2; do  # the two builds alternated
    run verify-timeline $rep
    timeout -k 10 120 tools/verify_timeline 3 64 >> "$OUT/verify_timeline.jsonl" 2>> "$OUT/verify_timeline.err"
    run verify-timeline-kp $rep
    timeout -k 10 120 tools/verify_timeline_kp 3 64 >> "$OUT/verify_timeline_kp.jsonl" 2>> "$OUT/verify_timeline_kp.err"
  done
fi
if [[ $STEPS == *deferred_ab* ]]; then
  # config-1 DEFERRED vs verify off: background PCIe reads, recv-ring footprint (tools/deferred_ab.cpp)
  run deferred-ab
  timeout -k 10 300 tools/deferred_ab 5 > "$OUT/deferred_ab.jsonl" 2> "$OUT/deferred_ab.err"
  # the same with as many HIP hardware queues as connections (one connection's verify never queues behind another's)
  run deferred-ab-8q
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 tools/deferred_ab 5 > "$OUT/deferred_ab_8q.jsonl" 2> "$OUT/deferred_ab_8q.err"
fi
if [[ $STEPS == *serial_ab* ]]; then
  # roofline leg: one graph of all K rotations (default) against K replays of a one-rotation graph, alternated
  for rep in 1 2 3; do
    for g in 0 1; do
      run serial-ab $rep $g
      timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --serial-graph-rotations $g \
        >> "$OUT/serial_ab.jsonl" 2>> "$OUT/serial_ab.err"
    done
  done
fi
run done
