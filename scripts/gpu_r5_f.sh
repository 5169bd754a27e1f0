#!/bin/bash
# Round 5, GPU call F (final build): the zero-copy entry trace back on the flat exchange, the
# full-size W=4 / W=8 shared-GPU bench rehearsals (one hardware queue per rank) and the driver's
# smoke(); the whole GPU suite is call G (scripts/gpu_r5_g.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash scripts/gpu_steps.sh \
  "fltrace2|240|python -u scripts/ipc_phase_trace.py --world 2 --mib 16 --iters 20 --modes zc --algo ipc" \
  "flab2|300|python -u scripts/dyn_bench.py --world 2 --mib 1,4,16,64 --algos 'ipc,ipc_dyn'" \
  "bench_w4|400|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 4 --steps 20 --warmup 5" \
  "bench_w8|500|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 8 --steps 20 --warmup 5" \
  "smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke()'"
