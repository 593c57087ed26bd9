#!/bin/bash
# round-2 session-4: parity of the split param_grad, step A/B (param_grad split x LayerNorm
# reductions deferred to the side stream), dW GEMM K-step / occupancy variants (kbench)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=hic-gnn_amd/hicgat
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "fullsize or overlapped or train_step or dense" -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/g_tests.log 2>&1; rc=$?; tail -3 gpurun_out/g_tests.log; [ $rc -le 1 ] || exit $rc
for rep in 1 2; do
for pg in 0 1; do
  for ln in 0 1; do
    HICGAT_PG_SPLIT=$pg HICGAT_LN_SIDE=$ln timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/g_pg${pg}_ln${ln}.json 2> gpurun_out/g_pg${pg}_ln${ln}.err || exit $?
    echo "pg_split=$pg ln_side=$ln $(python -c "import json;d=json.loads(open('gpurun_out/g_pg${pg}_ln${ln}.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['median_ms_per_step'],4))")"
  done
done
done
timeout -k 10 300 python tools/kbench.py --libs $L/libhicgat.so,$L/libhicgat_gk32.so,$L/libhicgat_gk32o2.so --only "gemm_dw_512x512#f32,gemm_dw_densea#f32,gemm_fwd_512#f32,gemm_dx_densea#f32" --reps 20 > gpurun_out/g_kb_gemm.txt 2>&1 || exit $?
cat gpurun_out/g_kb_gemm.txt
