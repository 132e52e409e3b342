# full GPU suite, then smoke + default bench, then a rocprofv3 kernel-trace run of the bench
cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_full.txt 2>&1 || { tail -30 gpurun_out/pytest_gpu_full.txt; exit 1; }
tail -2 gpurun_out/pytest_gpu_full.txt
bash scripts/full_check.sh || exit 1
