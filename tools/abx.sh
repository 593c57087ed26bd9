#!/bin/bash
# usage: abx.sh tag "ENV1=a ENV2=b" ...   (each argument one environment set; "X=1" = default)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; T=$1; shift
for E in "$@"; do
  env $E timeout -k 10 180 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/${T}_abx.json 2> gpurun_out/${T}_abx.err || exit $?
  echo "abx: $E $(python -c "import json;d=json.loads(open('gpurun_out/${T}_abx.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['median_ms_per_step'],4))")"
done
