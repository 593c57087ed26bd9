#!/bin/bash
# A/B: persistent source pass at 0 (full grid) / 3 / 4 / 5 workgroups per CU, side work FIFO vs
# largest-first, synth-20000 graph-replayed bench; prints ms_per_step / median per configuration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1; do
for w in 0 2 3 4; do
  for o in fifo size; do
    HICGAT_SRC_WGS=$w HICGAT_SIDE_ORDER=$o timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab_w${w}_${o}.json 2> gpurun_out/ab_w${w}_${o}.err || exit $?
    echo "wgs=$w order=$o $(python -c "import json,sys;d=json.loads(open('gpurun_out/ab_w${w}_${o}.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['median_ms_per_step'],4))")"
  done
done
done
