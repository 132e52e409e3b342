cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
run() {  # $1 = tag, rest = counters
  tag=$1; shift
  (cd /tmp && NNGP_SWEEP=${MODE:-launch} timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc/$tag -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing > $GRAFT_REPO_ROOT/gpurun_out/pmc/$tag.log 2>&1)
  echo "$tag rc=$?"
}
run fetch FETCH_SIZE && run write WRITE_SIZE && run tcc TCC_HIT_sum TCC_MISS_sum && run sq SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES && run ta TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE
ls gpurun_out/pmc/*/
