#!/bin/bash
# Round 5, GPU call U: the shared-device workgroup cap, wider sweep (W = 2 / 4 / 8; static and dyn).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
G="PDCC_TEST_SHARED_GRID"
bash scripts/gpu_steps.sh \
  "u_w2|400|python -u scripts/dyn_bench.py --world 2 --mib 1,4,16,64,256,1024 --iters 15 --algos 'ipc,ipc;$G=191,ipc;$G=224,ipc;$G=254,ipc_dyn,ipc_dyn;$G=191'" \
  "u_w4|400|python -u scripts/dyn_bench.py --world 4 --mib 1,4,16,64,256,1024 --iters 15 --algos 'ipc,ipc;$G=95,ipc;$G=112,ipc;$G=126,ipc_dyn,ipc_dyn;$G=95,ipc_dyn;$G=126'" \
  "u_w8|400|GPU_MAX_HW_QUEUES=1 python -u scripts/dyn_bench.py --world 8 --mib 1,16,256,1024 --iters 10 --algos 'ipc,ipc;$G=47,ipc;$G=55,ipc_dyn,ipc_dyn;$G=47'"
