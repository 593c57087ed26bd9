#!/bin/bash
# round-2 session-4: split-K target around the 256 default (192 / 256 / 384), step A/B x3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
for b in 192 256 384; do
  HICGAT_DW_BLOCKS=$b timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/r.json 2> gpurun_out/r.err || exit $?
  echo "r: dw_blocks=$b $(python -c "import json;d=json.loads(open('gpurun_out/r.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['median_ms_per_step'],4))")"
done
done
