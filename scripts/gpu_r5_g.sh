#!/bin/bash
# Round 5, GPU call G (final build): the whole GPU suite, as the driver runs it at round end.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
bash scripts/gpu_steps.sh "suite|1150|$T -m gpu tests/"
