cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for cfg in "HICGAT_GEMM_TALL=1" "HICGAT_GEMM_TALL=0" "HICGAT_LINATT=gemm"; do
  env $cfg timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
  echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profg -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/rocprof_graph.log 2>&1; echo "prof rc=$?"
