#!/bin/bash
# round-2 closing checks: synth-2000 bench with the MFMA roofline line; --gpus 2 on a 1-GPU box must
# fail loudly (exit 2 + an error JSON line)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload synth-2000 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/p_bench_synth2000.json 2> gpurun_out/p_bench_synth2000.err || exit $?
tail -1 gpurun_out/p_bench_synth2000.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], json.dumps(d['roofline']))"
timeout -k 10 120 python bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/p_gpus2.json 2> gpurun_out/p_gpus2.err; rc=$?
echo "--gpus 2 on one GPU: rc=$rc $(cat gpurun_out/p_gpus2.json)"
[ $rc -eq 2 ] || exit 1
