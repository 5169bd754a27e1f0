#!/bin/bash
# Round 5, GPU call E: the exchange's stores as global (not flat) instructions -- phase trace and
# per-call times at 1-256 MiB against call C's -- then the rest of the GPU suite after test_shared_gpu_world8 (which the
# previous call's run stopped in: 8 processes on one GPU, default hardware queues), the bench
# and multi-GPU test files, the full-size W=2 shared-GPU bench and a rocprofv3 kernel trace of the
# dynamic vs static all-reduce at 256 MiB (W=4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
REPO=$(pwd)
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
REST="world8 or ll_reduce_scatter_all_to_all or list_all_to_all_routing or ll_rooted_selftest or sync_collective_after_async or conformance or zero_copy or random_numerics or dynamic_allreduce or autotune_file or rccl_communicator or rccl_env_sweep or coalesced or phase_trace or capped_grid or mixing_async or mixed_async"
bash scripts/gpu_steps.sh \
  "zxtrace2|240|python -u scripts/ipc_phase_trace.py --world 2 --mib 16 --iters 20 --modes zc --algo ipc" \
  "zxab2|300|python -u scripts/dyn_bench.py --world 2 --mib 1,4,16,64 --algos 'ipc,ipc_dyn'" \
  "zxab4|300|python -u scripts/dyn_bench.py --world 4 --mib 1,4,16,64,256 --algos 'ipc,ipc_dyn'" \
  "suite_rest|900|$T -m gpu tests/test_backend_gpu.py -k '$REST'" \
  "suite_b|600|$T -m gpu tests/test_bench_launch.py tests/test_multi_gpu.py" \
  "bench_w2|300|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 2 --steps 10 --warmup 3" \
  "prof_dyn|300|cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/prof_dyn -o dyn -- python3 $REPO/scripts/dyn_bench.py --world 4 --mib 256 --iters 10 --algos ipc,ipc_dyn"
