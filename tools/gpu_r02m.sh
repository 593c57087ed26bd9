#!/bin/bash
# round-2 session-4: support pass fused into the background tile launch + resident loss seed:
# fused-loss parity tests, step A/B x3 against the previous build (HICGAT_LIB), rocprof trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=hic-gnn_amd/hicgat
timeout -k 10 400 python -u -m pytest tests/test_gpu_support.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "support or fullsize or fused or overlapped or train_loop or model" -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/m_tests.log 2>&1; rc=$?; tail -2 gpurun_out/m_tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
for lib in libhicgat_prev.so libhicgat.so; do
  HICGAT_LIB=$L/$lib timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/m.json 2> gpurun_out/m.err || exit $?
  echo "m: lib=$lib $(python -c "import json;d=json.loads(open('gpurun_out/m.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['median_ms_per_step'],4))")"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/m_prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/m_rocprof.log 2>&1 || exit $?
echo prof ok
