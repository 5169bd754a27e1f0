#!/bin/bash
# Round 5, GPU call AI (engine label of size-guarded gated calls): the guard test first, then the GPU suite and smoke().
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash scripts/gpu_steps.sh \
  "guard2|200|$T -m gpu tests/test_backend_gpu.py -k size_bit31" \
  "suite_g|1000|$T -m gpu tests/test_kernels_gpu.py tests/test_backend_gpu.py tests/test_bench_launch.py tests/test_multi_gpu.py" \
  "smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke()'"
