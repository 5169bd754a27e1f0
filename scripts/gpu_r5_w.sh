#!/bin/bash
# Round 5, GPU call W: 1 GiB zero-copy all_reduce phase trace at the new shared-device grid (W = 2 / 4 static).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
bash scripts/gpu_steps.sh \
  "w_tr2|200|python -u scripts/ipc_phase_trace.py --world 2 --mib 1024 --iters 10 --modes zc --algo ipc" \
  "w_tr4|200|python -u scripts/ipc_phase_trace.py --world 4 --mib 1024 --iters 10 --modes zc --algo ipc"
