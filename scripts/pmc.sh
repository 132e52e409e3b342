# Separate rocprofv3 --pmc passes over a short bench (1 chain), counters of
# the sweep kernel summarised per dispatch.
cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
run() {  # $1 = tag, rest = counters
  tag=$1; shift
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $ROOTDIR/gpurun_out/pmc/$tag -o run -- python3 $ROOTDIR/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-single-chain --chains ${CHAINS:-1} > $ROOTDIR/gpurun_out/pmc/$tag.log 2>&1)
  echo "$tag rc=$?"
}
run fetch FETCH_SIZE && run write WRITE_SIZE && run tcc TCC_HIT_sum TCC_MISS_sum && run ea TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum && run sq SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES && python3 scripts/pmc_summary.py gpurun_out/pmc sweep_color
