#!/bin/bash
# Round 5, GPU call AH (last build): full-size shared-GPU rehearsals at odd world sizes (W = 3 / 5 / 6 / 7).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
bash scripts/gpu_steps.sh \
  "bench_w3|300|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 3 --steps 10 --warmup 3" \
  "bench_w5|300|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 5 --steps 10 --warmup 3" \
  "bench_w6|300|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 6 --steps 10 --warmup 3" \
  "bench_w7|300|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 7 --steps 10 --warmup 3"
