#!/bin/bash
# Round 5, GPU call O: the W = 5 bf16 all-gather at 2 GiB per rank that stalls -- which part of the
# gated zero-copy path waits (device-side exchange on / off, 1 vs 2 GiB, W = 4 at 2 GiB).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
P="python -u scripts/ag_probe.py --engines ipc --iters 2 --timeout 20 --verbose"
bash scripts/gpu_steps.sh \
  "o_w5_2g|120|$P --world 5 --mib 2048 --env PDCC_LOG_LEVEL=3" \
  "o_w5_2g_nozx|120|$P --world 5 --mib 2048 --env PDCC_IPC_ZX=0" \
  "o_w5_1g|120|$P --world 5 --mib 1024" \
  "o_w4_2g|120|$P --world 4 --mib 2048" \
  "o_w5_2g_sync|120|$P --world 5 --mib 2048 --env PDCC_IPC_ZC_ASYNC=0"
