# SQ counters of the factor kernel (scripts/factor_prof.py), one pass.
cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd); export TMPDIR=/tmp
rm -rf gpurun_out/fpmc; mkdir -p gpurun_out/fpmc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $ROOTDIR/gpurun_out/fpmc/sq -o run -- python3 $ROOTDIR/scripts/factor_prof.py "$@" > $ROOTDIR/gpurun_out/fpmc/sq.log 2>&1) || exit 1
f=$(find gpurun_out/fpmc/sq -name "*counter_collection.csv" | head -1)
python3 - "$f" > gpurun_out/fpmc/summary.txt <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0]
    if "factor" not in k:
        continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    n = max(cnt[(k, c)] for c in d)
    print(k, "dispatches", n)
    for c, v in sorted(d.items()):
        print(f"  {c:24s} {v / n:16.0f}")
PY
cat gpurun_out/fpmc/summary.txt
