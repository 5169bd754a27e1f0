#!/bin/bash
# rocprofv3 kernel-trace + stats of the kernel microbench and of a 2-rank
# shared-GPU IPC run (our collective kernels). Summaries land in gpurun_out/prof*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/prof_kern" -o kb -- \
  python3 "$REPO/scripts/kernel_bench.py" > "$REPO/gpurun_out/prof_kern.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/prof_ipc" -o ipc -- \
  python3 "$REPO/scripts/ipc_demo.py" > "$REPO/gpurun_out/prof_ipc.log" 2>&1 || exit $?
echo profile-done
