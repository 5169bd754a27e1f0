#!/bin/bash
# Round 5, GPU call P: which bf16 all-gather sizes stall the zero-copy exchange (W = 2, one GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
P="python -u scripts/ag_probe.py --engines ipc --iters 1 --timeout 15 --verbose --world 2"
bash scripts/gpu_steps.sh \
  "p_1024|90|$P --mib 1024" \
  "p_2048|90|$P --mib 2048 --env PDCC_LOG_LEVEL=3" \
  "p_2046|90|$P --mib 2046" \
  "p_2050|90|$P --mib 2050" \
  "p_3072|90|$P --mib 3072" \
  "p_4096|90|$P --mib 4096"
