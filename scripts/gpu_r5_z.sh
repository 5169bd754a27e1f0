#!/bin/bash
# Round 5, GPU call Z: items per workgroup of the dynamic all_reduce (PDCC_IPC_DYN, default 3) at the new
# shared-device grid -- fewer, larger items mean fewer release fences (block 0: ~8 us per published item at W = 2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
bash scripts/gpu_steps.sh \
  "z_w2|300|python -u scripts/dyn_bench.py --world 2 --mib 16,64,256,1024 --iters 15 --algos 'ipc,ipc_dyn@1,ipc_dyn@2,ipc_dyn@3,ipc_dyn@6'" \
  "z_w4|300|python -u scripts/dyn_bench.py --world 4 --mib 16,64,256,1024 --iters 15 --algos 'ipc,ipc_dyn@1,ipc_dyn@2,ipc_dyn@3,ipc_dyn@6'" \
  "z_w8|300|GPU_MAX_HW_QUEUES=1 python -u scripts/dyn_bench.py --world 8 --mib 16,256,1024 --iters 10 --algos 'ipc,ipc_dyn@1,ipc_dyn@2,ipc_dyn@3'"
