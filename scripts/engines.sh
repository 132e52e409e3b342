#!/bin/bash
# GPU parity suite (all sweep engines), then the headline bench per engine.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-700} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -15 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
for eng in ${ENGINES:-tiles colors}; do
  NNGP_ENGINE=$eng timeout -k 10 400 python bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline --mcmc-iters ${MCMC:-0} ${BENCH_ARGS} > gpurun_out/bench_$eng.json 2> gpurun_out/bench_$eng.err
  rc=$?; echo "== $eng rc=$rc"; cat gpurun_out/bench_$eng.json | cut -c1-600; tail -3 gpurun_out/bench_$eng.err
  [ $rc -eq 0 ] || exit $rc
done
