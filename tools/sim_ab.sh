cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
for L in libhicgat libhicgat_gl8 libhicgat_nolds libhicgat; do for P in 8 2; do
  HICGAT_LIB=$PWD/hic-gnn_amd/hicgat/$L.so timeout -k 10 200 python bench.py --simulate-world $P --sim-rank 0 --dist-mode xagg --steps 50 --warmup 5 > gpurun_out/simab_${L}_$P.json 2> gpurun_out/simab_${L}_$P.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/simab_${L}_$P.json').read().strip().splitlines()[-1]);print('$L P=$P rank0', round(d['simulated']['rank_ms'][0],4), round(d['simulated']['rank_median_ms'][0],4))"
done; done
