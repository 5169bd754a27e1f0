#!/bin/bash
# Round 5, GPU call S: where a 1 GiB zero-copy all_reduce goes now (W = 2 static, W = 4 static and dyn),
# block 0's phase trace with per-block stamps, on the exchange-block build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
bash scripts/gpu_steps.sh \
  "s_tr2|200|python -u scripts/ipc_phase_trace.py --world 2 --mib 1024 --iters 10 --modes zc --algo ipc" \
  "s_tr4|200|python -u scripts/ipc_phase_trace.py --world 4 --mib 1024 --iters 10 --modes zc --algo ipc" \
  "s_tr4d|200|python -u scripts/ipc_phase_trace.py --world 4 --mib 1024 --iters 10 --modes zc --algo ipc_dyn"
