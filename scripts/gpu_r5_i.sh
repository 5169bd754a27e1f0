#!/bin/bash
# Round 5, GPU call I: isolated autotune runs -- the race probe again (W = 4, 1 GiB copy
# collectives), the autotuner / conformance GPU tests, and the full-size W=4 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash scripts/gpu_steps.sh \
  "race4|400|python -u scripts/race_probe.py --world 4 --mib 1024 --iters 5" \
  "tests_tune|600|$T -m gpu tests/test_backend_gpu.py -k 'autotune or conformance'" \
  "bench_w4|400|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 4 --steps 20 --warmup 5"
