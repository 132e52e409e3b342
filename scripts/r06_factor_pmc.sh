#!/bin/bash
# round 6: factor kernel A/B (one-lane vs 16-lane groups) + parity, counter list, and the tile
# sweep's request-size and instruction PMC passes (only counters the box lists)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/pmc6
ROOTDIR=$(pwd)
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "lane_groups" > gpurun_out/r06_factor_lanes_tests.txt 2>&1 || { tail -30 gpurun_out/r06_factor_lanes_tests.txt; exit 1; }
tail -2 gpurun_out/r06_factor_lanes_tests.txt
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTDIR/gpurun_out/prof_factor -o run -- python3 $ROOTDIR/scripts/factor_lanes_ab.py > $ROOTDIR/gpurun_out/r06_factor_lanes_ab.txt 2>&1) || { tail -20 gpurun_out/r06_factor_lanes_ab.txt; exit 1; }
tail -9 gpurun_out/r06_factor_lanes_ab.txt
f=$(find gpurun_out/prof_factor -name "*kernel_stats.csv" | head -1); grep -i "factor" "$f" | cut -c1-220
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $ROOTDIR/gpurun_out/pmc6/counters.txt 2>&1); echo "list rc=$?"
grep -o "TCC_[A-Z0-9_]*\|SQ_[A-Z0-9_]*" gpurun_out/pmc6/counters.txt | sort -u > gpurun_out/pmc6/names.txt; wc -l gpurun_out/pmc6/names.txt
pick() { for c in "$@"; do grep -qx "$c" gpurun_out/pmc6/names.txt && printf "%s " "${c}_sum"; done; }
pick0() { for c in "$@"; do grep -qx "$c" gpurun_out/pmc6/names.txt && printf "%s " "$c"; done; }
run() {  # $1 tag, rest counters
  tag=$1; shift
  [ -z "$*" ] && { echo "$tag: no counters"; return 0; }
  echo "$tag: $*"
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $* --output-format csv -d $ROOTDIR/gpurun_out/pmc6/$tag -o run -- python3 $ROOTDIR/bench.py --steps 10 --warmup 10 --no-cpu-baseline --no-kernel-timing --no-single-chain --no-rebuild-calls --mcmc-iters 0 --sustained-s 0 > $ROOTDIR/gpurun_out/pmc6/$tag.log 2>&1)
  echo "$tag rc=$?"
}
run req $(pick TCC_BUBBLE TCC_EA0_RDREQ_32B TCC_EA0_RDREQ) && \
run sq $(pick0 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU) && \
run sq2 $(pick0 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC)
for t in req sq sq2; do f=gpurun_out/pmc6/$t/run_counter_collection.csv; [ -f $f ] && python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "sweep_tiles" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:28s} per dispatch {sum(v) / len(v):16.1f} ({len(v)})")
PY
done
exit 0
