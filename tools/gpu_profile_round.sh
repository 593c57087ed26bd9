# The per-round evidence run: GPU suite, smoke, default bench (with CPU baseline), rocprofv3 kernel
# stats of the same bench, two PMC passes (FETCH_SIZE, WRITE_SIZE) for the roofline traffic.
# usage: bash tools/gpu_profile_round.sh <tag>   (writes gpurun_out/<tag>_*)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${T}_pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_rocprof.log 2>&1 || exit $?
echo "prof ok"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/${T}_pmc_fetch -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --eager > gpurun_out/${T}_pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/${T}_pmc_write -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --eager > gpurun_out/${T}_pmc_write.log 2>&1 || exit $?
echo "pmc ok"
