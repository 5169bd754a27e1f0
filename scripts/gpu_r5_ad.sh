#!/bin/bash
# Round 5, GPU call AD: 16 MiB all_reduce at W = 2, static vs dynamic, block 0's phase trace (every dyn item is
# static there: 128 reduce + 128 copy items on 128 workgroups, structurally the static split).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
bash scripts/gpu_steps.sh \
  "ad_s|200|python -u scripts/ipc_phase_trace.py --world 2 --mib 16 --iters 20 --modes zc --algo ipc" \
  "ad_d|200|python -u scripts/ipc_phase_trace.py --world 2 --mib 16 --iters 20 --modes zc --algo ipc_dyn"
