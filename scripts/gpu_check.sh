#!/bin/bash
# One GPU session: parity tests, then (if they did not crash) a short bench,
# then (PROFILE=1) a rocprofv3 kernel trace of a short bench.  Every GPU step
# has its own time limit; a crash/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOTDIR=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
rc=0
if [ -z "${SKIP_TESTS}" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -30 gpurun_out/pytest_gpu.log
  ok $rc || { echo "pytest rc=$rc: stopping"; exit $rc; }
fi
brc=0
if [ -z "${SKIP_BENCH}" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py --steps ${STEPS:-100} --warmup 10 ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
  brc=$?
  cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
  [ $brc -eq 0 ] || { echo "bench rc=$brc: stopping"; exit $brc; }
fi
if [ -n "${PROFILE}" ]; then
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOTDIR/gpurun_out/prof" -o run -- \
      python3 "$ROOTDIR/bench.py" --steps 40 --warmup 10 --no-cpu-baseline ${PROF_ARGS} > "$ROOTDIR/gpurun_out/bench_prof.json" 2> "$ROOTDIR/gpurun_out/bench_prof.err")
  prc=$?
  echo "rocprof rc=$prc"; find gpurun_out/prof -name "*stats*" | head
  [ $prc -eq 0 ] || exit $prc
fi
exit $rc
