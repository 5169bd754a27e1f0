#!/bin/bash
# Round 5, GPU call AB (final build): the driver's round-end steps -- smoke(), bench.py at its defaults (N = 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
bash scripts/gpu_steps.sh \
  "smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench1|300|python -u bench.py"
