#!/bin/bash
# round 6: normals' log_unit + fma running sums (b) against the previous build (a), plus the parity tests they touch
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "normals or sweep or headline or tile" > gpurun_out/r06_valu_tests.txt 2>&1 || { tail -30 gpurun_out/r06_valu_tests.txt; exit 1; }
tail -2 gpurun_out/r06_valu_tests.txt
bash scripts/ab_so.sh 3 a b
