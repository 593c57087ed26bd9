#!/bin/bash
# A/B of the synth-2000 bench (200 steps, no CPU baseline), one line per environment assignment:
#   bash tools/ab_synth2000.sh "ENV=a" "ENV=b" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for E in "$@"; do
  env $E timeout -k 10 200 python bench.py --workload synth-2000 --steps 200 --warmup 10 --no-cpu-baseline \
    > gpurun_out/b2k.json 2> gpurun_out/b2k.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/b2k.json').read().strip().splitlines()[-1]);print('synth-2000 $E', round(d['ms_per_step'],4), round(d['median_ms_per_step'],4))"
done
