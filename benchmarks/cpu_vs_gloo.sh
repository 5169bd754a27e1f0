#!/bin/bash
# The reference's own data path (torch.distributed + Gloo, CPU tensors) vs this
# library's host transport on the same machine; BASELINE.md method.
cd "$(dirname "$0")/.."
OUT=${OUT:-benchmarks/results/cpu_vs_gloo.jsonl}
: > "$OUT"
for w in 2 4 8; do
  for b in gloo mi355x; do
    timeout -k 10 1800 python benchmarks/coll_bench.py --world $w --backend $b --device cpu \
      --sizes ${SIZES:-4,256M} --iters ${ITERS:-3} 2>/dev/null | grep '^{' >> "$OUT"
  done
done
