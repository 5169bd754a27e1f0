#!/bin/bash
# Round 5, GPU call AC: the shared-device grid test.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
bash scripts/gpu_steps.sh \
  "grid_test|200|python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_backend_gpu.py -k 'grid_widens or phase_trace_records'"
