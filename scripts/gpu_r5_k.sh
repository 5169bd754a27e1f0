#!/bin/bash
# Round 5, GPU call K: the whole GPU suite and smoke() on the exchange-block build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash scripts/gpu_steps.sh \
  "suite|1000|$T -m gpu tests/" \
  "smoke|300|python -u -c 'import __graft_entry__ as g; g.smoke()'"
