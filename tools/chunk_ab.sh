set -e
STAGES="tests" bash tools/gpu_check.sh
for c in 1 2 4; do HICGAT_SRC_CHUNKS=$c timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c$c.log 2>&1; done
