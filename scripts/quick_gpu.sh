#!/bin/bash
# Fast GPU loop: the tile-engine parity tests (K=..., default: sweep tests), then the headline bench variants (abv.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-400} python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mcmc.py -m gpu -x -q --timeout 200 --timeout-method thread -k "${K:-sweep or batched or headline or configs1 or lockstep}" > gpurun_out/pytest_quick.log 2>&1
  rc=$?; tail -4 gpurun_out/pytest_quick.log
  [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
bash scripts/abv.sh
