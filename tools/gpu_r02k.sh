#!/bin/bash
# round-2 session-4: param_grad stage 2 in 256-thread blocks; step A/B x3 over (HICGAT_SRC_WGS,
# HICGAT_DW_BLOCKS) at the new defaults; rocprof trace of the default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "overlapped or fullsize or train_loop" -m gpu -v -rf --timeout 200 --timeout-method thread > gpurun_out/k_tests.log 2>&1; rc=$?; tail -2 gpurun_out/k_tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
for cfg in "0 256" "3 256" "0 128" "3 128"; do
  set -- $cfg
  HICGAT_SRC_WGS=$1 HICGAT_DW_BLOCKS=$2 timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/k.json 2> gpurun_out/k.err || exit $?
  echo "k: wgs=$1 dw_blocks=$2 $(python -c "import json;d=json.loads(open('gpurun_out/k.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['median_ms_per_step'],4))")"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/k_prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/k_rocprof.log 2>&1 || exit $?
echo prof ok
