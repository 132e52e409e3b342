#!/bin/bash
# HIP API + kernel trace of the bench's MCMC iterations (3 chains, 1e6/m15; diagnostic):
# which host calls sit in the device's idle gaps -> gpurun_out/prof_api/, gpurun_out/mcmc_api_gaps.txt
cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
(cd /tmp && timeout -k 10 400 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d $ROOTDIR/gpurun_out/prof_api -o run -- python3 $ROOTDIR/scripts/mcmc_prof.py --no-cprofile > $ROOTDIR/gpurun_out/prof_api.log 2>&1) || { tail -20 gpurun_out/prof_api.log; exit 1; }
python3 scripts/api_gaps.py gpurun_out/prof_api > gpurun_out/mcmc_api_gaps.txt && cat gpurun_out/mcmc_api_gaps.txt
