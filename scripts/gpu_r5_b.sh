#!/bin/bash
# Round 5, GPU call B: the dynamic protocol's fixed cost (verdict r4 Next #5) -- phase trace of
# ipc_dyn at 16 MiB (block 0's claim / ready / departure totals) and the dyn_bench A/B of the
# round-5 claim loop and control-word placement against round 4's -- then the new GPU tests again,
# the world-1 RCCL rehearsal, and the full-size W=8 shared-GPU bench rehearsal on one hardware
# queue per rank (verdict r4 Next #6).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
bash scripts/gpu_steps.sh \
  "dyntrace2|240|python -u scripts/ipc_phase_trace.py --world 2 --mib 16 --iters 20 --modes zc --algo ipc_dyn" \
  "dyntrace4|240|python -u scripts/ipc_phase_trace.py --world 4 --mib 16 --iters 20 --modes zc --algo ipc_dyn" \
  "dynab2|300|python -u scripts/dyn_bench.py --world 2 --mib 16,64,256 --algos ipc,ipc_dyn,ipc_dyn~8,ipc_dyn~24" \
  "dynab4|300|python -u scripts/dyn_bench.py --world 4 --mib 16,64,256 --algos ipc,ipc_dyn,ipc_dyn~8,ipc_dyn~24" \
  "dynag4|240|python -u scripts/dyn_bench.py --world 4 --mib 16,64,256 --coll all_gather --algos ipc,ipc_dyn" \
  "tests_new|600|$T tests/test_backend_gpu.py -k 'conformance or dynamic_allreduce or mixed_async or capped_grid or autotune or phase_trace'" \
  "rehearsal|450|$T --timeout 430 tests/test_bench_launch.py -k rehearsal -m gpu" \
  "bench_w8|500|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 8 --steps 10 --warmup 3"
