set -e
for r in 1 2; do for v in 1 0; do HICGAT_LN_SIDE=$v timeout -k 10 300 python bench.py --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/ln_$v.$r.log 2>&1; done; done
