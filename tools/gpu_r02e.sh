#!/bin/bash
# source-pass loads in flight (HICGAT_SRC_U 4 vs 8) x persistent grid x side issue order, synth-20000
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=hic-gnn_amd/hicgat
for cfg in "libhicgat.so 0 fifo" "libhicgat.so 2 size" "libhicgat_u8.so 2 size" "libhicgat_u8.so 3 size" "libhicgat_u8.so 0 fifo" "libhicgat.so 0 fifo" "libhicgat_u8.so 2 size" "libhicgat_u8.so 4 size"; do
  set -- $cfg
  HICGAT_LIB=$L/$1 HICGAT_SRC_WGS=$2 HICGAT_SIDE_ORDER=$3 timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/b_u.json 2>/dev/null || exit $?
  echo "$1 wgs=$2 order=$3 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_u.json) $(grep -o '"median_ms_per_step": [0-9.]*' gpurun_out/b_u.json)"
done
