#!/bin/bash
# round-2 session-4: big dW GEMMs on a side stream of their own (HICGAT_SIDE_BIG threshold in
# multiply-adds: 0 = off, 1e9 = the 256- and 512-wide tail blocks, 3e9 = the 512-wide only) and the
# dW split target (HICGAT_DW_BLOCKS), step A/B x2; rocprof trace of the 1e9 form
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "overlapped or wgrad" -m gpu -v -rf --timeout 200 --timeout-method thread > gpurun_out/i_tests.log 2>&1; rc=$?; tail -2 gpurun_out/i_tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
for cfg in "0 512" "1e9 512" "3e9 512" "1e9 256"; do
  set -- $cfg
  HICGAT_SIDE_BIG=$1 HICGAT_DW_BLOCKS=$2 timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/i_$1_$2.json 2> gpurun_out/i_$1_$2.err || exit $?
  echo "side_big=$1 dw_blocks=$2 $(python -c "import json;d=json.loads(open('gpurun_out/i_$1_$2.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['median_ms_per_step'],4))")"
done
done
HICGAT_SIDE_BIG=1e9 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/i_prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/i_rocprof.log 2>&1 || exit $?
echo prof ok
