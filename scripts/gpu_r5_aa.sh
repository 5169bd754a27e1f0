#!/bin/bash
# Round 5, GPU call AA: launch size of gated zero-copy calls (launcher.cpp kGateChunk = 256 MiB; a 1 GiB
# all_reduce runs as 4 launches, ~26 us apart) -- PDCC_TEST_GATE_CHUNK A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
C="PDCC_TEST_GATE_CHUNK"
bash scripts/gpu_steps.sh \
  "aa_w2|300|python -u scripts/dyn_bench.py --world 2 --mib 256,512,1024 --iters 15 --algos 'ipc,ipc;$C=536870912,ipc;$C=1073741824'" \
  "aa_w4|300|python -u scripts/dyn_bench.py --world 4 --mib 256,512,1024 --iters 15 --algos 'ipc_dyn,ipc_dyn;$C=536870912,ipc_dyn;$C=1073741824,ipc;$C=1073741824'" \
  "aa_w8|300|GPU_MAX_HW_QUEUES=1 python -u scripts/dyn_bench.py --world 8 --mib 256,1024 --iters 10 --algos 'ipc_dyn,ipc_dyn;$C=1073741824'"
