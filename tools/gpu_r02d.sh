#!/bin/bash
# side-stream placement A/B on synth-20000 (gather path): issue order x param_grad stream, and the
# persistent source-pass grid; rocprof trace of the old arrangement (fifo, param_grad on main)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "fifo 0 0" "size 0 0" "fifo 1 0" "size 1 0" "fifo 0 4" "size 0 4" "fifo 0 0" "size 0 2"; do
  set -- $cfg
  HICGAT_SIDE_ORDER=$1 HICGAT_PG_SIDE=$2 HICGAT_SRC_WGS=$3 timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/b_side.json 2>/dev/null || exit $?
  echo "order=$1 pg_side=$2 wgs=$3 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_side.json) $(grep -o '"median_ms_per_step": [0-9.]*' gpurun_out/b_side.json)"
done
HICGAT_SIDE_ORDER=fifo HICGAT_PG_SIDE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_fifo -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/p_fifo.log 2>&1 || exit $?
echo done
