#!/bin/bash
# Round 5, GPU call V (size-dependent shared-device cap build): per-call times at the new default, the
# full-size W = 2 / 4 / 8 bench rehearsals, then the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash scripts/gpu_steps.sh \
  "v_w2|300|python -u scripts/dyn_bench.py --world 2 --mib 1,4,16,64,256,1024 --iters 15 --algos 'ipc,ipc_dyn'" \
  "v_w4|300|python -u scripts/dyn_bench.py --world 4 --mib 1,4,16,64,256,1024 --iters 15 --algos 'ipc,ipc_dyn'" \
  "v_w8|300|GPU_MAX_HW_QUEUES=1 python -u scripts/dyn_bench.py --world 8 --mib 1,16,256,1024 --iters 10 --algos 'ipc,ipc_dyn'" \
  "bench_w2|300|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 2 --steps 20 --warmup 5" \
  "bench_w4|300|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 4 --steps 20 --warmup 5" \
  "bench_w8|400|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 8 --steps 20 --warmup 5" \
  "suite_v|1000|$T -m gpu tests/test_kernels_gpu.py tests/test_backend_gpu.py tests/test_bench_launch.py tests/test_multi_gpu.py"
