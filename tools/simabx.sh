#!/bin/bash
# usage: simabx.sh tag "ENV1=a ENV2=b" ...   rank 0 of the simulated 8-rank xagg step under each environment set
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; T=$1; shift
for E in "$@"; do
  env $E timeout -k 10 240 python bench.py --simulate-world 8 --sim-rank 0 --dist-mode xagg --steps 100 --warmup 5 \
    > gpurun_out/${T}_simabx.json 2> gpurun_out/${T}_simabx.err || exit $?
  echo "simabx: $E $(python -c "import json;d=json.loads(open('gpurun_out/${T}_simabx.json').read().strip().splitlines()[-1]);print([round(v,4) for v in d['simulated']['rank_ms']], [round(v,4) for v in d['simulated']['rank_median_ms']])")"
done
