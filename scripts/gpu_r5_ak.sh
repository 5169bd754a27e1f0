#!/bin/bash
# Round 5, GPU call AK: the GPU suite on the exact last build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
bash scripts/gpu_steps.sh \
  "suite_last|1000|python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_backend_gpu.py tests/test_bench_launch.py tests/test_multi_gpu.py"
