cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_support.py tests/test_gpu_fullsize.py > gpurun_out/pytest_adhoc.log 2>&1 || { tail -40 gpurun_out/pytest_adhoc.log; exit 1; }
grep -E "support nnz|mse dense|passed|failed" gpurun_out/pytest_adhoc.log | cut -c1-250
for f in 1 0 1 0; do
HICGAT_TRUTH_SUPPORT=$f timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
echo "$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profg -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/rocprof_graph.log 2>&1; echo "prof rc=$?"
