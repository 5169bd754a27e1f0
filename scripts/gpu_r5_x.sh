#!/bin/bash
# Round 5, GPU call X: non-temporal stores (PDCC_TEST_IPC_FLAGS bit 1: gather copy, bit 2: reduce stores)
# in the static and dynamic zero-copy all_reduce at the new shared-device grid: does the per-item
# release fence of the dynamic protocol pay for L2 write-backs?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
bash scripts/gpu_steps.sh \
  "x_w2|300|python -u scripts/dyn_bench.py --world 2 --mib 16,256,1024 --iters 15 --algos 'ipc,ipc~4,ipc~6,ipc_dyn,ipc_dyn~4,ipc_dyn~6'" \
  "x_w4|300|python -u scripts/dyn_bench.py --world 4 --mib 16,256,1024 --iters 15 --algos 'ipc,ipc~6,ipc_dyn,ipc_dyn~4,ipc_dyn~6'"
