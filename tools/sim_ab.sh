#!/bin/bash
# A/B of the simulated sharded step (bench.py --simulate-world P --sim-rank 0, xagg form): one line
# per (environment assignment, P), rank 0's ms/step mean and median.
#   bash tools/sim_ab.sh "ENV=a ENV2=b" "ENV=c" ...      (P in SIM_PS, default "8 4")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for E in "$@"; do for P in ${SIM_PS:-8 4}; do
  env $E timeout -k 10 200 python bench.py --simulate-world $P --sim-rank 0 --dist-mode xagg --steps 50 --warmup 5 \
    > gpurun_out/simab_$P.json 2> gpurun_out/simab_$P.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/simab_$P.json').read().strip().splitlines()[-1]);print('$E', 'P=$P rank0', round(d['simulated']['rank_ms'][0],4), round(d['simulated']['rank_median_ms'][0],4))"
done; done
