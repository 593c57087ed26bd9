cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "HICGAT_LINL_MAIN=0" "HICGAT_LINL_MAIN=1" "HICGAT_LINL_MAIN=0" "HICGAT_LINL_MAIN=1" "HICGAT_DEFER=0"; do
env $cfg timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench.log)"
done
HICGAT_LINL_MAIN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profg -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/rocprof_graph.log 2>&1; echo "prof rc=$?"
