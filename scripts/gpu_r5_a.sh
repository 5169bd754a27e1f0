#!/bin/bash
# Round 5, GPU call A: the new / changed GPU tests, the RCCL rehearsal of the bench, the W=8
# queue time-slicing probe (default queues vs GPU_MAX_HW_QUEUES=1) and a full-size W=4
# shared-GPU bench (the autotuner now races the IPC variants above 4 MiB without RCCL).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
bash scripts/gpu_steps.sh \
  "tests_new|600|$T tests/test_backend_gpu.py -k 'conformance or dynamic_allreduce or mixed_async or capped_grid or autotune'" \
  "rehearsal|450|$T --timeout 430 tests/test_bench_launch.py -k rehearsal -m gpu" \
  "slicing_default|300|python -u scripts/queue_slicing_probe.py --world 8 --iters 10" \
  "slicing_q1|300|python -u scripts/queue_slicing_probe.py --world 8 --iters 10 --queues 1" \
  "bench_w4|400|PDCC_BENCH_SMALL=0 python -u bench.py --gpus 4 --steps 10 --warmup 3"
