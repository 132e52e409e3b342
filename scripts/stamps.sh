cd $GRAFT_REPO_ROOT
NNGP_PROBE=9 NNGP_DBG_OUT=gpurun_out/stamps.bin timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-single-chain --chains 1 --no-kernel-timing > gpurun_out/stamps.json 2> gpurun_out/stamps.err || exit 1
python3 scripts/stamps_summary.py gpurun_out/stamps.bin 31
