#!/bin/bash
# Round 5, GPU call L: rocprofv3 kernel trace of gated zero-copy all-reduces on the exchange-block
# build (grid = data blocks + 1), and the full-size W=2 bench on the final build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
REPO=$(pwd)
bash scripts/gpu_steps.sh \
  "prof_xb|300|cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/prof_xb -o xb -- python3 $REPO/scripts/dyn_bench.py --world 2 --mib 16 --iters 10 --algos ipc" \
  "bench_w2|300|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 2 --steps 20 --warmup 5"
