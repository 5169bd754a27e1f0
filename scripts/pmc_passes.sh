#!/bin/bash
# Byte-reconciling PMC passes over scripts/pmc_k1_big.py (verdict r3 Next #7): the raw TCC->EA
# request counters by size next to rocprof's derived FETCH_SIZE / WRITE_SIZE, one counter set per
# run (gfx950: at most 4 TCC counters per pass), each run under its own hard time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT="$REPO/gpurun_out/pmc4"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
passes=(
  "rd:TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
  "wr:TCC_BUBBLE_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
  "fetch:FETCH_SIZE"
  "write:WRITE_SIZE"
)
for p in "${passes[@]}"; do
  tag=${p%%:*}
  set=${p#*:}
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/$tag" -o pmc -- \
    python3 "$REPO/scripts/pmc_k1_big.py" > "$OUT/$tag.log" 2>&1 || { echo "pass $tag failed: $?"; exit 1; }
done
python3 "$REPO/scripts/summarize_pmc.py" "$OUT" > "$OUT/summary.md" && echo pmc-done
