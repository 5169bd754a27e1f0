#!/bin/bash
# Round 5, GPU call Y: the dynamic all_reduce at W = 2 (1 GiB, 256 MiB launches) -- where its time goes
# (block 0's dyn totals), next to W = 4 where it wins.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
bash scripts/gpu_steps.sh \
  "y_tr2d|200|python -u scripts/ipc_phase_trace.py --world 2 --mib 1024 --iters 10 --modes zc --algo ipc_dyn" \
  "y_tr4d|200|python -u scripts/ipc_phase_trace.py --world 4 --mib 1024 --iters 10 --modes zc --algo ipc_dyn"
