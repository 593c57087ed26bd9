#!/bin/bash
# A/B of the simulated sharded step in bench.py's default "auto" form (rank 0, P in SIM_PS):
#   SIM_PS="2" bash tools/sim_ab_mode.sh "ENV=a" "ENV=b" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for E in "$@"; do for P in ${SIM_PS:-2}; do
  env $E timeout -k 10 200 python bench.py --simulate-world $P --sim-rank 0 --steps 50 --warmup 5 \
    > gpurun_out/simabm_$P.json 2> gpurun_out/simabm_$P.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/simabm_$P.json').read().strip().splitlines()[-1]);print('$E', 'P=$P', d['simulated']['mode'], 'rank0', round(d['simulated']['rank_ms'][0],4), round(d['simulated']['rank_median_ms'][0],4))"
done; done
