#!/bin/bash
# Round 5, GPU call AF (final build): smoke(), the full-size W = 2 / 4 / 8 shared-GPU rehearsals, the GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash scripts/gpu_steps.sh \
  "smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_w2|300|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 2 --steps 20 --warmup 5" \
  "bench_w4|300|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 4 --steps 20 --warmup 5" \
  "bench_w8|400|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 8 --steps 20 --warmup 5" \
  "suite_f|1000|$T -m gpu tests/test_kernels_gpu.py tests/test_backend_gpu.py tests/test_bench_launch.py tests/test_multi_gpu.py"
