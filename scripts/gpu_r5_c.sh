#!/bin/bash
# Round 5, GPU call C: the dynamic protocols' item size (PDCC_IPC_DYN_MIN_ROWS 8 / 16 / 32 / 64)
# against the static protocol, the new GPU tests again, and the full-size W=8 shared-GPU bench
# rehearsal (one hardware queue per rank; the ZeRO row capped to what fits one GPU); the call number
# taken before the arguments are staged vs after (PDCC_TEST_IPC_FLAGS=32, round-4 order).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
MR="ipc,ipc_dyn;PDCC_IPC_DYN_MIN_ROWS=8,ipc_dyn,ipc_dyn;PDCC_IPC_DYN_MIN_ROWS=32,ipc_dyn;PDCC_IPC_DYN_MIN_ROWS=64"
bash scripts/gpu_steps.sh \
  "dynmr2|300|python -u scripts/dyn_bench.py --world 2 --mib 16,64,256 --algos '$MR'" \
  "dynmr4|300|python -u scripts/dyn_bench.py --world 4 --mib 16,64,256 --algos '$MR'" \
  "dynmr4ag|300|python -u scripts/dyn_bench.py --world 4 --mib 16,64,256 --coll all_gather --algos '$MR'" \
  "dyntrace2|240|python -u scripts/ipc_phase_trace.py --world 2 --mib 16 --iters 20 --modes zc --algo ipc_dyn" \
  "seqtrace2|240|python -u scripts/ipc_phase_trace.py --world 2 --mib 16 --iters 20 --modes zc --algo ipc" \
  "seqtrace2_old|240|python -u scripts/ipc_phase_trace.py --world 2 --mib 16 --iters 20 --modes zc --algo ipc --test-flags 32" \
  "seqab2|300|python -u scripts/dyn_bench.py --world 2 --mib 1,4,16,64 --algos 'ipc,ipc~32'" \
  "seqab4|300|python -u scripts/dyn_bench.py --world 4 --mib 1,4,16,64 --algos 'ipc,ipc~32'" \
  "tests_new|600|$T tests/test_backend_gpu.py -k 'conformance or dynamic_allreduce or mixed_async or capped_grid or autotune or phase_trace'" \
  "bench_w8|500|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 8 --steps 10 --warmup 3"
