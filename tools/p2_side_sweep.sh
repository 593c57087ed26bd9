# P = 2 sweep of the xagg side branch's grouped dW workgroup target (rank 0 of the simulated 2-rank step); results: profiles/r06zh_ab_side_wgs_P2.txt
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for rep in 1 2; do
for W in 256 128 192 384 512; do
  HICGAT_XAGG_SIDE_WGS=$W timeout -k 10 240 python bench.py --simulate-world 2 --sim-rank 0 --dist-mode xagg --steps 100 --warmup 5 > gpurun_out/r06zh_p2_$W.json 2> gpurun_out/r06zh_p2_$W.err || exit $?
  echo "P=2 side_wgs=$W $(python -c "import json;d=json.loads(open('gpurun_out/r06zh_p2_$W.json').read().strip().splitlines()[-1]);print([round(v,4) for v in d['simulated']['rank_ms']], [round(v,4) for v in d['simulated']['rank_median_ms']])")"
done
done
