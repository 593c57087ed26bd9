set -e
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/occ_new.$r.log 2>&1
  HICGAT_LIB=hic-gnn_amd/hicgat/libhicgat_base.so timeout -k 10 300 python bench.py --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/occ_base.$r.log 2>&1
done
