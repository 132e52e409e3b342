#!/bin/bash
# GPU tests touched by the r-in-global default (configs[4] tests, RG parity)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 600 --timeout-method thread \
  -k "configs or global or residency" > gpurun_out/rg_tests.log 2>&1 || { tail -30 gpurun_out/rg_tests.log; exit 1; }
tail -2 gpurun_out/rg_tests.log
