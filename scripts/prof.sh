# rocprofv3 kernel trace (+stats) of short bench runs: 1 chain and 3 chains.
cd $GRAFT_REPO_ROOT
ROOTDIR=$(pwd)
export TMPDIR=/tmp
for C in 1 3; do
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/gpurun_out/prof_c$C" -o run -- \
      python3 "$ROOTDIR/bench.py" --steps 40 --warmup 10 --no-cpu-baseline --no-single-chain --chains $C > "$ROOTDIR/gpurun_out/prof_c$C.json" 2> "$ROOTDIR/gpurun_out/prof_c$C.err") || exit 1
  f=$(find gpurun_out/prof_c$C -name "*kernel_stats.csv" | head -1)
  echo "== C=$C $f"; head -12 "$f" | cut -c1-220
done
