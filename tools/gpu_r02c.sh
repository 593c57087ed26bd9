#!/bin/bash
# persistent source pass A/B: bench at HICGAT_SRC_WGS = 0 (full grid), 3..6 WGs per CU; parity of the
# persistent form; a rocprof trace of the best guess
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
HICGAT_SRC_WGS=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -v -rf -s --timeout 250 --timeout-method thread -k "backward" > gpurun_out/src_wgs_parity.log 2>&1; rc=$?; tail -3 gpurun_out/src_wgs_parity.log; [ $rc -le 1 ] || exit $rc
for w in 0 4 0 3 5 6 2; do
  HICGAT_SRC_WGS=$w timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/b_wgs$w.json 2>/dev/null || exit $?
  echo "wgs=$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_wgs$w.json) $(grep -o '"median_ms_per_step": [0-9.]*' gpurun_out/b_wgs$w.json)"
done
HICGAT_SRC_WGS=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_wgs4 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/p_wgs4.log 2>&1 || exit $?
echo done
