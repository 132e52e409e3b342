cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for k in 1 2; do timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b200_$k.json 2> gpurun_out/b200_$k.err || { tail -5 gpurun_out/b200_$k.err; exit 1; }; python3 -c "import json; d=json.loads(open('gpurun_out/b200_$k.json').read().strip().splitlines()[-1]); print(round(d['value']), d['secondary'])"; done
