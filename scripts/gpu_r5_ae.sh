#!/bin/bash
# Round 5, GPU call AE (strided dyn items build): dyn tests first, then static vs dyn (strided, the new
# default) vs dyn~64 (contiguous items, the previous layout) for all_reduce / all_gather / reduce_scatter.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash scripts/gpu_steps.sh \
  "ae_tests|600|$T -m gpu tests/test_backend_gpu.py -k 'dyn or dynamic or numerics or conformance or autotune'" \
  "ae_w2|300|python -u scripts/dyn_bench.py --world 2 --mib 1,16,64,256,1024 --iters 15 --algos 'ipc,ipc_dyn,ipc_dyn~64'" \
  "ae_w4|300|python -u scripts/dyn_bench.py --world 4 --mib 1,16,64,256,1024 --iters 15 --algos 'ipc,ipc_dyn,ipc_dyn~64'" \
  "ae_w8|300|GPU_MAX_HW_QUEUES=1 python -u scripts/dyn_bench.py --world 8 --mib 16,256,1024 --iters 10 --algos 'ipc,ipc_dyn,ipc_dyn~64'" \
  "ae_ag4|300|python -u scripts/dyn_bench.py --world 4 --coll all_gather --mib 16,64,256 --iters 15 --algos 'ipc,ipc_dyn,ipc_dyn~64'" \
  "ae_rs4|300|python -u scripts/dyn_bench.py --world 4 --coll reduce_scatter --mib 16,64,256 --iters 15 --algos 'ipc,ipc_dyn,ipc_dyn~64'"
