#!/bin/bash
# round 6: branch-free products in the workgroup-batch own draw (h: 1-2 chains, configs[4]'s 2+1 groups)
# against e; parity subset; configs[4]'s per-GPU share on each build
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_warm_calls.py tests/test_gpu_shard.py > gpurun_out/r06_h_tests.txt 2>&1 || { tail -30 gpurun_out/r06_h_tests.txt; exit 1; }
tail -2 gpurun_out/r06_h_tests.txt
bash scripts/ab_so.sh 2 e h || exit 1
cp lib/libnngp.so lib/libnngp_cur.so
for v in e h; do
  cp lib/libnngp_$v.so lib/libnngp.so
  timeout -k 10 400 python -u scripts/chain_groups_bench.py 1250000 20 3 60 > gpurun_out/r06_cg_$v.txt 2>&1 || { tail -5 gpurun_out/r06_cg_$v.txt; cp lib/libnngp_cur.so lib/libnngp.so; exit 1; }
  echo "$v:"; grep '"arm"' gpurun_out/r06_cg_$v.txt | cut -c1-200
done
cp lib/libnngp_cur.so lib/libnngp.so
