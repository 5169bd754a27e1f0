#!/bin/bash
# Round 5, GPU call N: the bf16 ZeRO all-gather row that ran the W = 5/6/7 rehearsals' extras past
# their deadline, engine by engine (scripts/ag_probe.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
bash scripts/gpu_steps.sh \
  "ag5|300|python -u scripts/ag_probe.py --world 5 --mib 2048 --engines ipc,ipc_dyn,ipc_staged,auto" \
  "ag7|300|python -u scripts/ag_probe.py --world 7 --mib 1024 --engines ipc,ipc_dyn,ipc_staged,auto"
