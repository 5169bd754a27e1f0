#!/bin/bash
# GPU validation run for gpurun: each GPU step under its own time limit; a test
# FAILURE (pytest rc 1) does not stop the chain, a crash/timeout/abort does.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/steps.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2> >(tee -a "gpurun_out/$name.err" >&2)
  local rc=$?
  echo "rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    smoke) step smoke 300 python __graft_entry__.py ;;
    kern) step kern 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread ;;
    backend) step backend 900 python -u -m pytest tests/test_backend_gpu.py -x -v --timeout 300 --timeout-method thread ;;
    gputests) step gputests 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    graphbench) step graphbench 300 python scripts/graph_bench.py ;;
    graphbench1) GRAPH_BENCH_MODE=rccl1 step graphbench1 300 python scripts/graph_bench.py ;;
    bench1) step bench1 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench2dbg) PDCC_BENCH_SMALL=1 PDCC_LOG_LEVEL=2 PDCC_BENCH_DEBUG_S=150 step bench2dbg 240 \
        python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29534 bench.py --gpus 2 --steps 3 --warmup 1 --bytes 67108864 ;;
    kprof) step kprof 600 python scripts/kernel_bench.py ;;
    benchdeadline) PDCC_BENCH_SMALL=1 PDCC_BENCH_EXTRAS_S=4 step benchdeadline 300 python -m torch.distributed.run \
        --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --steps 3 \
        --warmup 1 --bytes 67108864 ;;
    profile) step profile 1500 bash scripts/profile.sh ;;
    pmc) PDCC_PMC_ONLY=1 step pmc 600 bash scripts/profile.sh ;;
    trace) PDCC_TRACE_ONLY=1 step trace 900 bash scripts/profile.sh ;;
    k2sweep) step k2sweep 300 python scripts/k2_sweep.py ;;
    bench2self) PDCC_BENCH_SMALL=1 step bench2self 600 python bench.py --gpus 2 --steps 3 --warmup 1 --bytes 67108864 ;;
    churn) step churn 300 python scripts/group_churn.py ;;
    graphprobe) step graphprobe 300 python scripts/graph_probe.py ;;
    graphrt) step graphrt 200 python scripts/graph_rt_probe.py ;;
    graphprobe_q1) GPU_MAX_HW_QUEUES=1 step graphprobe_q1 300 python scripts/graph_probe.py ;;
    graphprof) step graphprof 400 bash -c 'cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$0/gpurun_out/prof_graph" -o g -- python3 "$0/scripts/graph_bench.py"' "$(pwd)" ;;
    zcbench) step zcbench 400 python scripts/zc_bench.py ;;
    zcbench4) step zcbench4 400 python scripts/zc_bench.py --world 4 --sizes 4M,64M ;;
    zcprobe) step zcprobe 120 python scripts/ipc_buffer_probe.py ;;
    zctest) step zctest 600 python -u -m pytest tests/test_backend_gpu.py -x -v --timeout 300 --timeout-method thread \
        -k "zero_copy or selftest or bulk or golden" ;;
    zcprof) step zcprof 500 bash -c 'cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$0/gpurun_out/prof_zc" -o zc -- python3 "$0/scripts/zc_bench.py" --sizes 64M --iters 8 --modes zc' "$(pwd)" ;;
    stgprof) step stgprof 500 bash -c 'cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$0/gpurun_out/prof_stg" -o stg -- python3 "$0/scripts/zc_bench.py" --sizes 64M --iters 8 --modes staged' "$(pwd)" ;;
    conf) step conf 900 python -u -m pytest tests/test_backend_gpu.py -x -v --timeout 300 --timeout-method thread \
        -k "conformance or list_all_to_all or ll_reduce_scatter or world8 or async or autotune" ;;
    zcasync) step zcasync 600 python -u -m pytest tests/test_backend_gpu.py -x -v --timeout 300 --timeout-method thread \
        -k "zero_copy or zc or churn or conformance or push or async" ;;
    zerobench) step zerobench 600 python scripts/zero_bench.py ;;
    zcdebug) step zcdebug 150 python scripts/zc_debug.py zero_copy --world 3 --dump-s 60 \
        --env PDCC_ALGO=ipc PDCC_IPC_ZC_CACHE=4 PDCC_IPC_1SHOT_MAX=256K ;;
    atsdebug) step atsdebug 150 python scripts/zc_debug.py async_then_sync --world 2 --dump-s 40 \
        --env PDCC_ALGO=ipc ;;
    zcasyncbench) step zcasyncbench 300 python scripts/zc_async_bench.py ;;
    churntrace) step churntrace 400 bash -c 'cd /tmp && TMPDIR=/tmp rocprofv3 --hip-trace --stats --output-format csv \
        -d "$0/gpurun_out/prof_churn" -o churn_%pid% -- python3 "$0/scripts/zc_async_bench.py" --churn' "$(pwd)" ;;
    hostpath) step hostpath 300 python scripts/host_path_bench.py ;;
    hostpathtr) step hostpathtr 300 python scripts/host_path_bench.py --trace ;;
    hostpathinl) step hostpathinl 300 python scripts/host_path_bench.py --trace --env PDCC_IPC_ZC_ASYNC=0 ;;
    hostpathspin0) step hostpathspin0 300 python scripts/host_path_bench.py --trace --env PDCC_XCHG_SPIN_US=0 ;;
    cpuinfo) step cpuinfo 30 bash -c 'cat /sys/fs/cgroup/cpu.max 2>&1; cat /sys/fs/cgroup/cpuset.cpus.effective 2>&1; nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)))"' ;;
    hostprof) step hostprof 400 bash -c 'cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$0/gpurun_out/prof_host" -o hp_%pid% -- python3 "$0/scripts/host_path_bench.py" --calls 400' "$(pwd)" ;;
    tgdebug) step tgdebug 150 python scripts/zc_debug.py two_groups --world 2 --dump-s 40 --env PDCC_ALGO=ipc ;;
    k1sweep) step k1sweep 300 python scripts/k1_sweep.py ;;
    gpuA) step gpuA 1100 python -u -m pytest tests/test_backend_gpu.py -v --timeout 300 --timeout-method thread ;;
    gpuB) step gpuB 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
        --deselect tests/test_backend_gpu.py ;;
    gpuA2) step gpuA2 600 python -u -m pytest tests/test_backend_gpu.py -v --timeout 300 --timeout-method thread \
        -k "world8 or list_all_to_all or conformance or ll_reduce_scatter" ;;
    bench2shared) PDCC_BENCH_SMALL=1 step bench2shared 600 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 \
        --bytes 67108864 ;;
  esac
done
