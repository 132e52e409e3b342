#!/bin/bash
# default build (185 VGPRs, 2 waves/SIMD) vs waves_per_eu(3) and (4) builds placed in lib/alt/ by hand (one-off; not kept)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in default w3 w4; do
  lib=lib/libnngp.so; [ $v != default ] && lib=lib/alt/$v.so
  NNGP_LIB=$lib NNGP_AB_N=1250000 NNGP_AB_M=20 timeout -k 10 200 python -u scripts/ab_env.py 3 50 2 "$v:" > gpurun_out/wpe_share_$v.txt 2>&1 || { tail -20 gpurun_out/wpe_share_$v.txt; exit 1; }
  grep rep gpurun_out/wpe_share_$v.txt
done
for v in default w3 w4; do
  lib=lib/libnngp.so; [ $v != default ] && lib=lib/alt/$v.so
  NNGP_LIB=$lib NNGP_AB_N=10000000 NNGP_AB_M=20 timeout -k 10 280 python -u scripts/ab_env.py 3 20 1 "$v:" > gpurun_out/wpe_1e7_$v.txt 2>&1 || { tail -20 gpurun_out/wpe_1e7_$v.txt; exit 1; }
  grep rep gpurun_out/wpe_1e7_$v.txt
done
