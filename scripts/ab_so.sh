#!/bin/bash
# A/B of two builds of the extension in one GPU call: ab_so.sh <tag> <so_a> <so_b> <rounds> -- <cmd...>
# runs <cmd> with build A, then build B, <rounds> times (interleaved), output in gpurun_out/ab_<tag>_<A|B><k>.log;
# stops at the first failing step (no retries)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=$1; a=$2; b=$3; rounds=$4; shift 5
SO=pytorch_distributed_collective_communication_amd/_C.cpython-310-x86_64-linux-gnu.so
for k in $(seq 1 "$rounds"); do
  for v in A B; do
    src=$a; [ "$v" = B ] && src=$b
    cp "$src" "$SO" || exit 1
    echo "=== $tag $v$k ($src)"
    timeout -k 10 300 "$@" > "gpurun_out/ab_${tag}_${v}${k}.log" 2>&1 || { echo "rc=$? at $v$k"; exit 1; }
    tail -2 "gpurun_out/ab_${tag}_${v}${k}.log"
  done
done
