cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bw.json 2> gpurun_out/bw.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/bw.json').read().strip().splitlines()[-1]);print('steps20 mean', round(d['ms_per_step'],4), 'median', round(d['median_ms_per_step'],4))"
done
