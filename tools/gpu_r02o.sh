#!/bin/bash
# round-2 session-4: gradient zeroing beside the forward (HICGAT_ZG_SIDE): tests, step A/B x3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -k "graph or adam or captured or overlapped or replay or train_loop or train_step" -v -rf --timeout 300 --timeout-method thread > gpurun_out/o_tests.log 2>&1; rc=$?; tail -2 gpurun_out/o_tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
for z in 0 1; do
  HICGAT_ZG_SIDE=$z timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/o.json 2> gpurun_out/o.err || exit $?
  echo "o: zg_side=$z $(python -c "import json;d=json.loads(open('gpurun_out/o.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['median_ms_per_step'],4))")"
done
done
