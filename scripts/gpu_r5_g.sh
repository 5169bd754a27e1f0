#!/bin/bash
# Round 5, GPU call G (final build): the full-size W=8 shared-GPU bench rehearsal, then the whole GPU
# suite, as the driver runs it at round end.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash scripts/gpu_steps.sh \
  "bench_w8|300|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 8 --steps 20 --warmup 5" \
  "suite|1000|$T -m gpu tests/"
