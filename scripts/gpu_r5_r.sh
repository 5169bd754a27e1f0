#!/bin/bash
# Round 5, GPU call R (size guard build): the guard's test, the W = 5 2 GiB all-gather probe, and the
# W = 5 / 6 / 7 full-size shared-GPU bench rehearsals whose extras stalled in call M.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash scripts/gpu_steps.sh \
  "guard_test|200|$T -m gpu tests/test_backend_gpu.py -k 'size_bit31 or epoch_wraps or device_exchange_selftest'" \
  "ag5g|200|python -u scripts/ag_probe.py --world 5 --mib 2048 --engines ipc,ipc_dyn,auto --timeout 30 --verbose" \
  "bench_w5|300|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 5 --steps 10 --warmup 3" \
  "bench_w6|300|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 6 --steps 10 --warmup 3" \
  "bench_w7|300|GPU_MAX_HW_QUEUES=1 PDCC_BENCH_SMALL=0 python -u bench.py --gpus 7 --steps 10 --warmup 3"
