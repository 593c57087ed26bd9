#!/bin/bash
# One gpurun call: GPU parity tests, smoke, a short bench and a rocprofv3 kernel-trace summary.
# Assertion failures (exit 1) do not stop the script; a crash, abort, fault or timeout does.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -n 25 "gpurun_out/$name.log" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc" >&2; exit $rc; fi
  return 0
}
STAGES=${STAGES:-"tests smoke bench prof"}
for s in $STAGES; do
  case $s in
    tests) run pytest_gpu 600 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread ;;
    tfast) run pytest_fast 300 python -u -m pytest tests/test_gpu_fast_paths.py -m gpu -v -rf --timeout 120 --timeout-method thread ;;
    benchx3) HICGAT_GEMM=auto run bench_x3 600 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline ;;
    dscc) run dscc 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k dscc_chr19 -s -v --timeout 240 --timeout-method thread ;;
    n2v) run n2v 300 python -u -m pytest tests/test_gpu_node2vec.py -m gpu -v -rf --timeout 180 --timeout-method thread ;;
    aux) run bench_aux 300 python tools/bench_aux.py ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS:---no-cpu-baseline} ;;
    benche) run bench_eager 600 python bench.py --steps ${STEPS:-20} --warmup 3 --eager --no-cpu-baseline ;;
    benchcpu) run bench_cpu 900 python bench.py ;;
    c2d) run debug_c2d 300 python tools/debug_c2d.py ;;
    kbench) run kbench 600 python tools/kbench.py --libs ${KLIBS:-hic-gnn_amd/hicgat/libhicgat.so} ;;
    kbench_nolds) HICGAT_PD_NOLDS=1 run kbench_nolds 600 python tools/kbench.py ;;
    prof)  run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
               python bench.py --steps 10 --warmup 2 --no-cpu-baseline --eager ;;
    pmc)   run pmc_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- \
               python bench.py --steps 3 --warmup 1 --no-cpu-baseline --eager &&
           run pmc_write 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- \
               python bench.py --steps 3 --warmup 1 --no-cpu-baseline --eager ;;
    pmcl2) run pmc_l2 600 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_l2 -o run --output-format csv -- \
               python bench.py --steps 3 --warmup 1 --no-cpu-baseline --eager ;;
  esac
done
