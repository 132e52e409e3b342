#!/bin/bash
# round 6: LDS counters of the tile sweep kernel (bank / address conflicts, unaligned stalls,
# bandwidth) at the bench workload, two separate --pmc passes (kernel-trace only)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/pmcl
ROOTDIR=$(pwd)
run() {  # $1 tag, rest counters
  tag=$1; shift
  echo "$tag: $*"
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $* --output-format csv -d $ROOTDIR/gpurun_out/pmcl/$tag -o run -- python3 $ROOTDIR/bench.py --steps 10 --warmup 10 --no-cpu-baseline --no-kernel-timing --no-single-chain --no-rebuild-calls --mcmc-iters 0 --sustained-s 0 > $ROOTDIR/gpurun_out/pmcl/$tag.log 2>&1)
  echo "$tag rc=$?"
}
run l1 SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_WAIT_INST_LDS SQ_LDS_DATA_FIFO_FULL && \
run l2 SQ_INSTS_LDS_STORE SQ_INSTS_LDS_STORE_BANDWIDTH SQ_LDS_CMD_FIFO_FULL SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INST_LEVEL_LDS SQ_WAVES SQ_ACTIVE_INST_LDS || exit 1
for t in l1 l2; do f=gpurun_out/pmcl/$t/run_counter_collection.csv; [ -f $f ] && python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "sweep_tiles" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:30s} per dispatch {sum(v) / len(v):16.1f} ({len(v)})")
PY
done
exit 0
