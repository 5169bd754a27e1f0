#!/bin/bash
# Round 5, GPU call AJ (after reverting the engine-label change): the zero-copy tests it broke, the guard test, smoke().
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash scripts/gpu_steps.sh \
  "zc_tests|400|$T -m gpu tests/test_backend_gpu.py -k 'zero_copy or size_bit31 or grid_widens'" \
  "smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke()'"
