#!/bin/bash
# Round 5, GPU call Q: the zero-copy stall's size rule -- 2-4 GiB stalls, 4 GiB does not: is it bit 31 of
# the exported allocation's size (5 GiB: clear, 6 GiB: set)?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
P="python -u scripts/ag_probe.py --engines ipc --iters 1 --timeout 15 --verbose --world 2"
bash scripts/gpu_steps.sh \
  "q_5120|90|$P --mib 5120" \
  "q_6144|90|$P --mib 6144" \
  "q_8192|90|$P --mib 8192"
