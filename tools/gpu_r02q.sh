#!/bin/bash
# round-2 session-4: the tall 160x128 GEMM only for problems of >= 400 tiles (block 2's 256-wide
# GEMMs, 250 tiles, on the 64x128 kernel instead): step A/B x3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
for t in 0 400; do
  HICGAT_TALL_MIN_TILES=$t timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/q.json 2> gpurun_out/q.err || exit $?
  echo "q: tall_min_tiles=$t $(python -c "import json;d=json.loads(open('gpurun_out/q.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['median_ms_per_step'],4))")"
done
done
