# per-phase timeline of the tile kernel (NNGP_PROBE=2) at 3 and 1 chains
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python scripts/timeline.py 1000000 15 3 10 > gpurun_out/r03_tl3.txt 2>&1 || exit 1
timeout -k 10 300 python scripts/timeline.py 1000000 15 1 10 > gpurun_out/r03_tl1.txt 2>&1 || exit 1
cat gpurun_out/r03_tl3.txt gpurun_out/r03_tl1.txt | grep -v amdgpu.ids
