#!/bin/bash
# round-2 session-4: Adam advances the device step count itself (ticket, no second launch):
# graph-replay / Adam tests, step A/B x3 against the previous build (HICGAT_LIB)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=hic-gnn_amd/hicgat
timeout -k 10 400 python -u -m pytest tests -m gpu -k "graph or adam or captured or overlapped or replay or train_loop or dist" -v -rf --timeout 300 --timeout-method thread > gpurun_out/n_tests.log 2>&1; rc=$?; tail -2 gpurun_out/n_tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
for lib in libhicgat_prev.so libhicgat.so; do
  HICGAT_LIB=$L/$lib timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/n.json 2> gpurun_out/n.err || exit $?
  echo "n: lib=$lib $(python -c "import json;d=json.loads(open('gpurun_out/n.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['median_ms_per_step'],4))")"
done
done
