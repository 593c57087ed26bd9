#!/bin/bash
# round-2 session-3 measurement call: kbench A/B (pairdist occupancy, tiled vs gather aggregation on
# both synthetic workloads), rocprof stats of synth-2000 with tiles on/off and synth-20000 (tiles off)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=hic-gnn_amd/hicgat
timeout -k 10 300 python tests/golden/make_n2v_chr19.py gpurun_out/n2v_chr19_1mb.npz || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiles.py -m gpu -v -rf -s --timeout 200 --timeout-method thread > gpurun_out/tiles.log 2>&1; rc=$?; tail -5 gpurun_out/tiles.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/kbench.py --libs $L/libhicgat.so,$L/libhicgat_pdo4.so --only pairdist_support,gat_agg_fwd_train,gat_agg_fwd_tiled,gat_agg_bwd_src --reps 10 > gpurun_out/kb_20k.txt 2>&1 || exit $?
cat gpurun_out/kb_20k.txt
timeout -k 10 300 python tools/kbench.py --workload synth-2000 --only gat_agg_fwd_train,gat_agg_fwd_tiled,gat_agg_bwd_src --reps 10 > gpurun_out/kb_2k.txt 2>&1 || exit $?
cat gpurun_out/kb_2k.txt
for t in 64 0; do
  HICGAT_TILE_MIN=$t timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_2k_$t -o run --output-format csv -- python bench.py --workload synth-2000 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/p_2k_$t.log 2>&1 || exit $?
done
HICGAT_TILE_MIN=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_20k -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/p_20k.log 2>&1 || exit $?
HICGAT_TILE_MIN=0 timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/b_20k.json 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*' gpurun_out/p_*.log gpurun_out/b_20k.json
