# smoke + default bench (the driver's round-end commands), outputs under gpurun_out/
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; rc=$?
cat gpurun_out/bench_default.json; tail -4 gpurun_out/bench_default.err; exit $rc
