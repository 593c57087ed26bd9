#!/bin/bash
# round-2 session-4: fused loss without d in the MSE-only path (w = 1 - t/d, (d - t)^2 = w^2 d^2):
# loss parity tests, step A/B x3 against the previous build (HICGAT_LIB)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
L=hic-gnn_amd/hicgat
timeout -k 10 500 python -u -m pytest tests -m gpu -k "support or fused or pairdist or loss or fullsize or train_loop or dscc or model or smoke" -v -rf --timeout 300 --timeout-method thread > gpurun_out/s_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s_tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
for lib in libhicgat_prev.so libhicgat.so; do
  HICGAT_LIB=$L/$lib timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/s.json 2> gpurun_out/s.err || exit $?
  echo "s: lib=$lib $(python -c "import json;d=json.loads(open('gpurun_out/s.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['median_ms_per_step'],4), d['final_loss'])")"
done
done
timeout -k 10 200 python tools/kbench.py --libs $L/libhicgat_prev.so,$L/libhicgat.so --only pairdist_support --reps 20 > gpurun_out/s_kb.txt 2>&1 || exit $?
cat gpurun_out/s_kb.txt | grep pairdist
