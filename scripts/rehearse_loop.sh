#!/bin/bash
# Diagnostic: repeat the 2-ranks-on-one-GPU bench rehearsal; each run dumps
# Python stacks (faulthandler) and exits if it is still running after 100 s.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_backend_gpu.py -q -k "two_ipc or golden" > gpurun_out/two_groups.log 2>&1; echo "tests rc=$?" | tee -a gpurun_out/loop.log
for i in 1 2 3; do
  echo "=== run $i" | tee -a gpurun_out/loop.log
  PDCC_BENCH_SMALL=1 PDCC_BENCH_DEBUG_S=100 timeout -k 10 140 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29600 + i)) bench.py --gpus 2 --steps 3 \
    --warmup 1 --bytes 67108864 > gpurun_out/loop_$i.log 2> gpurun_out/loop_$i.err
  rc=$?
  echo "rc=$rc" | tee -a gpurun_out/loop.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
