#!/bin/bash
# round-2 session-4: param_grad stage 2 with all partial loads in flight; side-work order A/B x3
# (fifo vs small_first: the GEMM-free reductions first, beside the gather); rocprof trace of small_first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "overlapped or fullsize" -m gpu -v -rf --timeout 200 --timeout-method thread > gpurun_out/l_tests.log 2>&1; rc=$?; tail -2 gpurun_out/l_tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
for o in fifo small_first; do
  HICGAT_SIDE_ORDER=$o timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/l.json 2> gpurun_out/l.err || exit $?
  echo "l: order=$o $(python -c "import json;d=json.loads(open('gpurun_out/l.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['median_ms_per_step'],4))")"
done
done
HICGAT_SIDE_ORDER=small_first timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/l_prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/l_rocprof.log 2>&1 || exit $?
echo prof ok
