#!/bin/bash
# round-2 session-4: side-work placement under the new defaults (DW 256, LN sums deferred):
# default vs HICGAT_PG_SIDE=1 vs HICGAT_LINL_MAIN=0 vs HICGAT_SIDE_BIG=3e9, step A/B x3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
for cfg in "X=0" "HICGAT_PG_SIDE=1" "HICGAT_LINL_MAIN=0" "HICGAT_SIDE_BIG=3e9"; do
  env $cfg timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/t.json 2> gpurun_out/t.err || exit $?
  echo "t: $cfg $(python -c "import json;d=json.loads(open('gpurun_out/t.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['median_ms_per_step'],4))")"
done
done
