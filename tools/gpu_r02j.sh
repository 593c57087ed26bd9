#!/bin/bash
# round-2 session-4: step A/B x3 over (HICGAT_SRC_WGS, HICGAT_SIDE_BIG, HICGAT_DW_BLOCKS), 200 steps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
for cfg in "0 0 512" "0 1e9 256" "3 0 512" "3 1e9 512" "0 0 256" "3 1e9 256"; do
  set -- $cfg
  HICGAT_SRC_WGS=$1 HICGAT_SIDE_BIG=$2 HICGAT_DW_BLOCKS=$3 timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/j.json 2> gpurun_out/j.err || exit $?
  echo "wgs=$1 side_big=$2 dw_blocks=$3 $(python -c "import json;d=json.loads(open('gpurun_out/j.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['median_ms_per_step'],4))")"
done
done
