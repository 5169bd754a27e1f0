#!/bin/bash
# Run GPU steps one after another: "name|timeout_s|command" arguments. A step that ends with a
# test/assertion failure (exit 1) does not stop the rest; a time limit (124/137), an abort
# (134), a segfault (139) or any other code does -- nothing more touches the GPU after that.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/steps
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; to=${rest%%|*}; cmd=${rest#*|}
  echo "[steps] $name (limit ${to}s): $cmd"
  # progress heartbeat (a quiet step, e.g. one long pytest case, is still bounded by its own limit)
  ( t=0; while sleep 60; do t=$((t + 60)); echo "[steps] $name running ${t}s" >> "gpurun_out/steps/$name.hb"; done ) &
  hb=$!
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/steps/$name.log" 2>&1
  rc=$?
  kill $hb 2>/dev/null; wait $hb 2>/dev/null
  echo "[steps] $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[steps] stopping after $name"; exit $rc; fi
done
echo "[steps] all done"
