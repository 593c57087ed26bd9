#!/bin/bash
# round-2 closing evidence: the per-round script (suite, smoke, bench + CPU baseline, rocprof stats,
# two PMC passes) at tag r02e, then the synth-2000 (configs[1]) bench and its rocprof stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_profile_round.sh r02e || exit $?
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload synth-2000 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/r02e_bench_synth2000.json 2> gpurun_out/r02e_bench_synth2000.err || exit $?
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r02e_bench_synth2000.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02e_prof2k -o run --output-format csv -- python bench.py --workload synth-2000 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r02e_rocprof2k.log 2>&1 || exit $?
echo prof2k ok
