#!/bin/bash
# the full GPU suite and the smoke (the driver's round-end commands) -> gpurun_out/pytest_gpu_full.txt, smoke.log
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1050 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_full.txt 2>&1 || { tail -30 gpurun_out/pytest_gpu_full.txt; exit 1; }
tail -2 gpurun_out/pytest_gpu_full.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; exit $rc
