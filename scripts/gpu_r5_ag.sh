#!/bin/bash
# Round 5, GPU call AG: rocprofv3 kernel trace of the last build's 1 GiB all_reduce with 8 ranks on one GPU
# (dynamic protocol, the rehearsal's adopted engine) and with 2 ranks (static): per-dispatch workgroups and times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
REPO=$(pwd)
bash scripts/gpu_steps.sh \
  "prof_w8|300|cd /tmp && TMPDIR=/tmp GPU_MAX_HW_QUEUES=1 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/prof_last -o w8 -- python3 $REPO/scripts/dyn_bench.py --world 8 --mib 1024 --iters 10 --algos ipc_dyn" \
  "prof_w2|300|cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/prof_last -o w2 -- python3 $REPO/scripts/dyn_bench.py --world 2 --mib 1024 --iters 10 --algos ipc"
