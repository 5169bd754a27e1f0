#!/bin/bash
# Round 5, GPU call T: workgroups per rank when ranks share the GPU (PDCC_TEST_SHARED_GRID; default 256 / W,
# plus the exchange block on gated launches) -- zero-copy all_reduce 16 / 256 / 1024 MiB, W = 2 and 4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
G="PDCC_TEST_SHARED_GRID"
bash scripts/gpu_steps.sh \
  "t_w2|400|python -u scripts/dyn_bench.py --world 2 --mib 16,256,1024 --iters 15 --algos 'ipc,ipc;$G=127,ipc;$G=120,ipc;$G=112,ipc;$G=96,ipc;$G=160,ipc;$G=192'" \
  "t_w4|400|python -u scripts/dyn_bench.py --world 4 --mib 16,256,1024 --iters 15 --algos 'ipc,ipc;$G=63,ipc;$G=56,ipc;$G=48,ipc;$G=80,ipc;$G=96,ipc_dyn,ipc_dyn;$G=63,ipc_dyn;$G=96'"
