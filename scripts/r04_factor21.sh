#!/bin/bash
# m = 20 factor: register-template BM = 21 (lib/) vs the scratch-array runtime kernel (altlib/, the previous build)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "factor_matches_oracle and 20" > gpurun_out/f21_tests.log 2>&1 || { tail -30 gpurun_out/f21_tests.log; exit 1; }
tail -1 gpurun_out/f21_tests.log
for lib in lib/libnngp.so altlib/libnngp_rt.so lib/libnngp.so; do
  NNGP_LIB=$ROOT$PWD/$lib timeout -k 10 300 python -u scripts/factor_time.py 1e6 20 2>&1 | tail -1 | sed "s|^|$lib: |" || exit 1
done
