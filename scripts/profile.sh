#!/bin/bash
# rocprofv3 kernel-trace + stats of the kernel microbench and of a 2-rank
# shared-GPU IPC run (our collective kernels). Summaries land in gpurun_out/prof*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
if [ "${PDCC_TRACE_ONLY:-0}" = 1 ]; then
  # tracing subsystem: roctx ranges per collective (PDCC_ROCTX=1) next to the
  # kernels they launch, and RCCL API trace of a world-1 RCCL communicator
  PDCC_ROCTX=1 timeout -k 10 600 rocprofv3 --marker-trace --kernel-trace --stats --summary --output-format csv \
    -d "$REPO/gpurun_out/trace_ipc" -o tr -- python3 "$REPO/scripts/ipc_demo.py" \
    > "$REPO/gpurun_out/trace_ipc.log" 2>&1 || exit $?
  PDCC_ROCTX=1 PDCC_WORLD1_LOCAL=0 PDCC_BENCH_EXTRAS=0 timeout -k 10 600 rocprofv3 --marker-trace --rccl-trace \
    --kernel-trace --stats --summary --output-format csv -d "$REPO/gpurun_out/trace_rccl1" -o tr -- \
    python3 "$REPO/bench.py" --gpus 1 --steps 10 --warmup 2 > "$REPO/gpurun_out/trace_rccl1.log" 2>&1 || exit $?
  echo trace-done
  exit 0
fi
if [ "${PDCC_PMC_ONLY:-0}" != 1 ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/prof_kern" -o kb -- \
  python3 "$REPO/scripts/kernel_bench.py" > "$REPO/gpurun_out/prof_kern.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$REPO/gpurun_out/prof_ipc" -o ipc -- \
  python3 "$REPO/scripts/ipc_demo.py" > "$REPO/gpurun_out/prof_ipc.log" 2>&1 || exit $?
fi
if [ "${PDCC_PMC:-1}" = 1 ]; then
  # hardware counters: one derived counter per run (FETCH_SIZE and WRITE_SIZE do
  # not fit one pass on gfx950), kernel-trace only alongside --pmc
  for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"; do
    tag=$(echo $set | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    timeout -k 10 150 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$REPO/gpurun_out/pmc_$tag" \
      -o pmc -- python3 "$REPO/scripts/pmc_k1.py" > "$REPO/gpurun_out/pmc_$tag.log" 2>&1 || exit $?
  done
fi
echo profile-done
