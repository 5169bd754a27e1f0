#!/bin/bash
# Round 5, GPU call D: the world-1 RCCL rehearsal of bench.py (record kept), the whole GPU test
# suite on this build, the full-size W=2 shared-GPU bench, and a rocprofv3 kernel trace of the
# dynamic vs static all-reduce at 256 MiB (W=4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
REPO=$(pwd)
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash scripts/gpu_steps.sh \
  "rehearsal_w1|400|PDCC_BENCH_RCCL_REHEARSAL=1 PDCC_BENCH_SMALL=1 python -u bench.py --gpus 1 --steps 5 --warmup 2 --bytes 67108864" \
  "suite_a|900|$T -m gpu tests/test_kernels_gpu.py tests/test_backend_gpu.py" \
  "suite_b|600|$T -m gpu tests/test_bench_launch.py tests/test_multi_gpu.py" \
  "bench_w2|300|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 2 --steps 10 --warmup 3" \
  "prof_dyn|300|cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/prof_dyn -o dyn -- python3 $REPO/scripts/dyn_bench.py --world 4 --mib 256 --iters 10 --algos ipc,ipc_dyn"
