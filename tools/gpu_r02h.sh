#!/bin/bash
# round-2 session-4: LDS-DMA weight-gradient kernel -- GEMM parity tests, kbench DMA vs VGPR-staged
# dW kernel, step A/B (HICGAT_WGRAD_DMA=1/0) x2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "gemm or wgrad or linear or overlapped or fullsize or dense or ln_relu" -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/h_tests.log 2>&1; rc=$?; tail -3 gpurun_out/h_tests.log; [ $rc -eq 0 ] || exit 1
for d in 1 0; do
  HICGAT_WGRAD_DMA=$d timeout -k 10 300 python tools/kbench.py --only "gemm_dw_512x512#f32,gemm_dw_densea#f32" --reps 20 > gpurun_out/h_kb_$d.txt 2>&1 || exit $?
  sed "s/^/dma=$d /" gpurun_out/h_kb_$d.txt | grep gemm
done
for rep in 1 2; do
for d in 1 0; do
    HICGAT_WGRAD_DMA=$d timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/h_d$d.json 2> gpurun_out/h_d$d.err || exit $?
    echo "wgrad_dma=$d $(python -c "import json;d=json.loads(open('gpurun_out/h_d$d.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['median_ms_per_step'],4))")"
done
done
HICGAT_WGRAD_DMA=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/h_prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/h_rocprof.log 2>&1 || exit $?
echo prof ok
