# Tile-shard checks (in-process groups, two processes on one GPU over HIP IPC); outputs in gpurun_out/
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_tile_shard.py tests/test_gpu_shard.py -m gpu > gpurun_out/shard_test.log 2>&1
tail -3 gpurun_out/shard_test.log
