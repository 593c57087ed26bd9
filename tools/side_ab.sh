set -e
for r in 1 2; do
  for cfg in "1 1" "1 0" "0 0"; do set -- $cfg
    HICGAT_OVERLAP=$1 HICGAT_SMALL_SIDE=$2 timeout -k 10 300 python bench.py --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/side_$1$2.$r.log 2>&1
  done
done
