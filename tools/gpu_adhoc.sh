cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in _old "" _nosb; do
for kind in fwd dx; do
HICGAT_LIB=$PWD/hic-gnn_amd/hicgat/libhicgat$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/profk$v$kind -o run --output-format csv -- python tools/gemm_loop.py $kind 20 > gpurun_out/gl.log 2>&1 || exit $?
echo "$v $kind $(grep tall gpurun_out/profk$v$kind/run_kernel_stats.csv | cut -d, -f 13-15)"
done
done
for v in _old "" _nosb _old ""; do
HICGAT_LIB=$PWD/hic-gnn_amd/hicgat/libhicgat$v.so timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench.log)"
done
