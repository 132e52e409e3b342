#!/bin/bash
# Request-size-resolved PMC passes (round 6): the sweep kernel at the bench workload and the
# known-byte calibration kernels, each counter set in its own rocprofv3 run (kernel trace only).
# HBM-side bytes = 128 x TCC_EA0_RDREQ_128B + 64 x _64B + 32 x _32B reads, and 64 x
# TCC_EA0_WRREQ_64B + 32 x (WRREQ - WRREQ_64B) writes (scripts/pmc_sizes_summary.py).
cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd); export TMPDIR=/tmp
D=gpurun_out/pmcs; mkdir -p $D
[ -x scripts/micro/calib ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/micro/calib.hip -o scripts/micro/calib || exit 1
run() {  # $1 tag, $2 bench|calib, rest counters
  tag=$1; kind=$2; shift 2
  if [ "$kind" = bench ]; then
    (cd /tmp && timeout -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $ROOTDIR/$D/$tag -o run -- python3 $ROOTDIR/bench.py --steps 10 --warmup 10 --no-cpu-baseline --no-kernel-timing --no-single-chain --no-rebuild-calls --mcmc-iters 0 --sustained-s 0 --chains ${CHAINS:-3} > $ROOTDIR/$D/$tag.log 2>&1)
  else
    (cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $ROOTDIR/$D/$tag -o run -- $ROOTDIR/scripts/micro/calib > $ROOTDIR/$D/$tag.log 2>&1)
  fi
  rc=$?; echo "$tag rc=$rc"; return $rc
}
R="TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum"
W="TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_UC_READ_REQ_sum"
run cal_r calib $R && run cal_w calib $W && run sw_r bench $R && run sw_w bench $W && \
run sw_f bench FETCH_SIZE && run sw_wr bench WRITE_SIZE && \
python3 scripts/pmc_sizes_summary.py $D ${KERNEL:-sweep_tiles} --json $D/summary.json --chains ${CHAINS:-3} --sweeps-per-dispatch 10
