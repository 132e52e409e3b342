# PMC passes (separate rocprofv3 --pmc runs, kernel-trace only): the sweep
# kernel at the bench workload, plus the known-byte calibration kernels.
cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
run() {  # $1 = tag, $2 = program kind, rest = counters
  tag=$1; kind=$2; shift 2
  if [ "$kind" = bench ]; then
    # warmup 10 + steps 10 = two calls of n_chromatic = 10 sweeps: every
    # dispatch of the tile kernel covers 10 sweeps
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $ROOTDIR/gpurun_out/pmc/$tag -o run -- python3 $ROOTDIR/bench.py --steps 10 --warmup 10 --no-cpu-baseline --no-kernel-timing --no-single-chain --mcmc-iters 0 --sustained-s 0 --chains ${CHAINS:-3} > $ROOTDIR/gpurun_out/pmc/$tag.log 2>&1)
  else
    (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $ROOTDIR/gpurun_out/pmc/$tag -o run -- $ROOTDIR/scripts/micro/calib > $ROOTDIR/gpurun_out/pmc/$tag.log 2>&1)
  fi
  echo "$tag rc=$?"
}
run cal_fetch calib FETCH_SIZE && run cal_write calib WRITE_SIZE && \
run fetch bench FETCH_SIZE && run write bench WRITE_SIZE && run tcc bench TCC_HIT_sum TCC_MISS_sum && \
run ea bench TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum && \
python3 scripts/pmc_summary.py gpurun_out/pmc ${KERNEL:-sweep_tiles} --json gpurun_out/pmc/summary.json --chains ${CHAINS:-3} --sweeps-per-dispatch ${SWEEPS:-10}
