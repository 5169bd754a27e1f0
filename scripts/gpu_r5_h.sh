#!/bin/bash
# Round 5, GPU call H: the autotuner's verdicts for the copy collectives at 1 GiB without RCCL
# (scripts/race_probe.py: race table + forced engines), W = 4 ranks on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
bash scripts/gpu_steps.sh \
  "race4|400|python -u scripts/race_probe.py --world 4 --mib 1024 --iters 5"
