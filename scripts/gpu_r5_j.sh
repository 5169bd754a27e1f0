#!/bin/bash
# Round 5, GPU call J: the exchange block (gated zero-copy launches run the device-side exchange in
# an extra workgroup) -- phase trace and per-call times against call F's, the dyn / static A/B at
# W = 4, and the full-size W=4 / W=8 shared-GPU rehearsals.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
bash scripts/gpu_steps.sh \
  "xbtrace2|240|python -u scripts/ipc_phase_trace.py --world 2 --mib 16 --iters 20 --modes zc --algo ipc" \
  "xbab2|300|python -u scripts/dyn_bench.py --world 2 --mib 1,4,16,64,256 --algos 'ipc,ipc_dyn'" \
  "xbab4|300|python -u scripts/dyn_bench.py --world 4 --mib 1,4,16,64,256 --algos 'ipc,ipc_dyn'" \
  "xbag4|300|python -u scripts/dyn_bench.py --world 4 --mib 1,16,256 --coll all_gather --algos 'ipc,ipc_dyn'" \
  "bench_w4|400|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 4 --steps 20 --warmup 5" \
  "bench_w8|400|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 8 --steps 20 --warmup 5"
