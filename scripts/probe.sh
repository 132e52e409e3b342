cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd); export TMPDIR=/tmp
for P in 0 4 5 6 7 8; do
  (cd /tmp && NNGP_PROBE=$P timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/gpurun_out/probe_$P" -o run -- \
     python3 "$ROOTDIR/bench.py" --steps 40 --warmup 10 --no-cpu-baseline --no-single-chain --chains 1 --no-kernel-timing > "$ROOTDIR/gpurun_out/probe_$P.json" 2> "$ROOTDIR/gpurun_out/probe_$P.err") || exit 1
  f=$(find gpurun_out/probe_$P -name "*kernel_stats.csv" | head -1)
  echo "probe $P: $(grep sweep_color $f | cut -d, -f3-7) value=$(python3 -c "import json;print(round(json.load(open('gpurun_out/probe_$P.json'))['value']))")"
done
