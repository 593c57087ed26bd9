#!/bin/bash
# One parametrised GPU run script (replaces the round-2 one-off gpu_r02*.sh files).
#
#   bash tools/gpu_run.sh <tag> <step> [<step> ...]      (outputs: gpurun_out/<tag>_*)
#
# steps (each under its own time limit; the script stops at the first failure):
#   tests        pytest -m gpu (whole GPU suite)
#   testsall     the same, test failures do not stop the later steps
#   probe_capture tools/capture_probe.py (legal order, then the round-5 slab order; put it LAST)
#   tests:<k>    pytest -m gpu -k <k>   (testsoft:<k>: test failures do not stop the later steps)
#   testenv:<env>:<k> pytest -m gpu -k <k> under an environment assignment
#   smoke        __graft_entry__.smoke()
#   bench        default bench.py (N = 1, synth-20000, with the CPU baseline)
#   bench2000    bench.py --workload synth-2000 --no-cpu-baseline
#   ab:<env>     bench.py 200 steps under the environment assignment(s) <env> (comma-separated; A/B lines "ab: ...")
#   ab2000:<env> the same on synth-2000 (400 steps)
#   prof         rocprofv3 --kernel-trace --stats of bench.py (20 steps, graph replay)
#   pmc_traffic  two PMC passes (FETCH_SIZE, WRITE_SIZE) of an eager bench -> <tag>_pmc_traffic.json
#   pmc_mfma     one PMC pass (MFMA busy cycles, F32 MFMA MOPs, GRBM_GUI_ACTIVE) -> <tag>_pmc_mfma.json
#   pmc_mfma2000 the same on synth-2000 (dense-tile MFMA aggregation)
#   pmc_mfma_sim the same for rank 0 of the simulated 8-rank xagg step
#   simrank      per-rank compute of the sharded step at P = 2, 4, 8 (bench.py --simulate-world; _ag: allgather
#                form, _xa: aggregate-first form, _au: bench.py's default "auto")
#   kb:<jobs>:<libs> tools/kbench.py A/B of the named kernel jobs over the listed library builds
#   simab:<env>  rank 0 of the simulated 8-rank xagg step (100 steps) under the environment assignment <env>
#   probe[:<env>] tools/xagg_probe.py: rank 0's xagg kernels one by one (optionally under <env>)
#   probegrads   the same plus the grouped parameter-gradient launches broken down by job
#   simprof      rocprofv3 kernel trace of rank 0's share of the simulated 8-rank step (+ one step's timeline)
#   align        the config-5 generalisation run (python -m hicgat.align) on chr19 1 mb -> 500 kb
#   n2v          node2vec feature study (tools/n2v_study.py): embedding structure + K=3000 dSCC per max_waves / seed
#   n2vfix       node2vec embeddings of chr19 1 mb, seeds 43 and 42 (fixtures for the oracle collapse check)
#   cli          the reference driver's flow (python -m hicgat.train) on chr19 1 mb with GPU node2vec
#                features, the default conversion sweep, 1000 steps each -> gpurun_out/<tag>_cli/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:?tag}
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
COMMIT=$(cat .commit 2>/dev/null || echo unknown)
for S in "$@"; do
  echo "== $S"
  case "$S" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread \
        > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc ;;
    testsall)
      # the whole suite; test failures (rc 1) do not stop the later steps, a crash / timeout does
      timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread \
        > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest_gpu.log; [ $rc -le 1 ] || exit $rc ;;
    probe_capture)
      # tools/capture_probe.py: the legal fork / join order, then the round-5 slab order (streams rule 2)
      # -- LAST in a call: the second may crash its process
      timeout -k 10 120 python tools/capture_probe.py ok > gpurun_out/${T}_capture_probe.txt 2>&1 || exit $?
      timeout -k 10 120 python tools/capture_probe.py rule2 >> gpurun_out/${T}_capture_probe.txt 2>&1; rc=$?
      echo "rule2 probe exit status $rc" >> gpurun_out/${T}_capture_probe.txt
      grep -v amdgpu.ids gpurun_out/${T}_capture_probe.txt ;;
    tests:*|testsoft:*)
      K=${S#tests:}; K=${K#testsoft:}
      timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf -s --timeout 300 --timeout-method thread -k "$K" \
        > gpurun_out/${T}_pytest_k.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest_k.log
      # testsoft: test failures (rc 1) do not stop the later steps; a crash / timeout does
      if [ "${S%%:*}" = testsoft ]; then [ $rc -le 1 ] || exit $rc; else [ $rc -eq 0 ] || exit $rc; fi ;;
    testenv:*)
      # testenv:<env assignment>:<k>  pytest -m gpu -k <k> under the environment assignment (e.g. HICGAT_LIB=...)
      R=${S#testenv:}; E=${R%%:*}; K=${R#*:}
      env $E timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf -s --timeout 300 --timeout-method thread -k "$K" \
        > gpurun_out/${T}_pytest_env.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest_env.log; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
      tail -1 gpurun_out/${T}_smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
      grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_bench.json ;;
    bench2000)
      timeout -k 10 300 python bench.py --workload synth-2000 --no-cpu-baseline > gpurun_out/${T}_bench_synth2000.json \
        2> gpurun_out/${T}_bench_synth2000.err || exit $?
      grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_bench_synth2000.json ;;
    ab:*)
      # ab:<env>[,<env>...]: one or more assignments, comma-separated
      E=${S#ab:}
      env ${E//,/ } timeout -k 10 180 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/${T}_ab.json \
        2> gpurun_out/${T}_ab.err || exit $?
      echo "ab: ${S#ab:} $(python -c "import json;d=json.loads(open('gpurun_out/${T}_ab.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['median_ms_per_step'],4))")" ;;
    ab2000:*)
      env ${S#ab2000:} timeout -k 10 180 python bench.py --workload synth-2000 --steps 400 --warmup 10 --no-cpu-baseline \
        > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err || exit $?
      echo "ab2000: ${S#ab2000:} $(python -c "import json;d=json.loads(open('gpurun_out/${T}_ab.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],4), round(d['median_ms_per_step'],4))")" ;;
    prof|prof:*)
      # prof:<env>[,<env>...]: under environment assignments (exported before rocprofv3: no launcher hop)
      if [ "$S" != prof ]; then E=${S#prof:}; for a in ${E//,/ }; do export "$a"; done; fi
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- \
        python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_rocprof.log 2>&1 || exit $?
      python tools/step_timeline.py gpurun_out/${T}_prof/run_kernel_trace.csv 10 > gpurun_out/${T}_step_timeline.txt || exit $?
      echo "prof ok" ;;
    pmc_traffic)
      timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/${T}_pmc_fetch -o run --output-format csv -- \
        python bench.py --steps 3 --warmup 1 --no-cpu-baseline --eager > gpurun_out/${T}_pmc_fetch.log 2>&1 || exit $?
      timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/${T}_pmc_write -o run --output-format csv -- \
        python bench.py --steps 3 --warmup 1 --no-cpu-baseline --eager > gpurun_out/${T}_pmc_write.log 2>&1 || exit $?
      python tools/pmc_traffic.py gpurun_out/${T}_pmc_fetch/run_counter_collection.csv \
        gpurun_out/${T}_pmc_write/run_counter_collection.csv gpurun_out/${T}_pmc_traffic.json synth-20000 \
        "rocprofv3 --kernel-trace --pmc FETCH_SIZE|WRITE_SIZE -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --eager" \
        "$COMMIT" > /dev/null || exit $?
      echo "pmc_traffic ok" ;;
    pmc_mfma|pmc_mfma2000)
      W=synth-20000; [ "$S" = pmc_mfma2000 ] && W=synth-2000
      timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
        -d gpurun_out/${T}_${S} -o run --output-format csv -- \
        python bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --eager > gpurun_out/${T}_${S}.log 2>&1 || exit $?
      python tools/pmc_mfma.py gpurun_out/${T}_${S}/run_counter_collection.csv x gpurun_out/${T}_${S}.json $W \
        "rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE -- python bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline --eager" \
        "$COMMIT" || exit $? ;;
    pmc_mfma_sim)
      # the MFMA counters of rank 0's share of the simulated 8-rank xagg step (graph replay, 3 steps)
      timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \
        -d gpurun_out/${T}_${S} -o run --output-format csv -- \
        python bench.py --simulate-world 8 --sim-rank 0 --dist-mode xagg --steps 3 --warmup 2 > gpurun_out/${T}_${S}.log 2>&1 || exit $?
      python tools/pmc_mfma.py gpurun_out/${T}_${S}/run_counter_collection.csv x gpurun_out/${T}_${S}.json sim-P8-rank0 \
        "rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE -- python bench.py --simulate-world 8 --sim-rank 0 --dist-mode xagg --steps 3 --warmup 2" \
        "$COMMIT" || exit $? ;;
    stamps)
      # per-phase cycles of the one-kernel tail forward / backward (diagnostic build libhicgat_stamps.so,
      # made on the CPU by `python tools/tail_stamps.py build`)
      timeout -k 10 300 python tools/tail_stamps.py run 8 > gpurun_out/${T}_stamps.txt 2>&1 || exit $?
      cat gpurun_out/${T}_stamps.txt | grep -v "^\[" ;;
    pmc_wait_sim)
      # where the waves of rank 0's share of the simulated 8-rank xagg step spend their cycles (one pass:
      # 8 SQ + 1 GRBM counters; WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES)
      timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
        -d gpurun_out/${T}_${S} -o run --output-format csv -- \
        python bench.py --simulate-world 8 --sim-rank 0 --dist-mode xagg --steps 3 --warmup 2 --no-bare > gpurun_out/${T}_${S}.log 2>&1 || exit $?
      python tools/pmc_summary.py gpurun_out/${T}_${S}/run_counter_collection.csv > gpurun_out/${T}_${S}.txt || exit $?
      echo "pmc_wait_sim ok" ;;
    simrank|simrank_ag|simrank_xa|simrank_au)
      M=slab; [ "$S" = simrank_ag ] && M=allgather; [ "$S" = simrank_xa ] && M=xagg; [ "$S" = simrank_au ] && M=auto
      for P in 2 4 8; do
        timeout -k 10 240 python bench.py --simulate-world $P --dist-mode $M --steps 50 --warmup 5 \
          > gpurun_out/${T}_simrank_${M}_P$P.json 2> gpurun_out/${T}_simrank_${M}_P$P.err || exit $?
        python -c "import json;d=json.loads(open('gpurun_out/${T}_simrank_${M}_P$P.json').read().strip().splitlines()[-1]);print('$M P=$P', [round(v,4) for v in d['simulated']['rank_ms']], round(d['simulated']['model_ms_per_step'],4))"
      done ;;
    simab:*)
      # A/B of rank 0's share of the simulated 8-rank xagg step under an environment assignment
      # (e.g. HICGAT_LIB=hic-gnn_amd/hicgat/libhicgat_db.so or HICGAT_GROUP_WGS=256)
      env ${S#simab:} timeout -k 10 240 python bench.py --simulate-world 8 --sim-rank 0 --dist-mode xagg --steps 100 \
        --warmup 5 > gpurun_out/${T}_simab.json 2> gpurun_out/${T}_simab.err || exit $?
      echo "simab: ${S#simab:} $(python -c "import json;d=json.loads(open('gpurun_out/${T}_simab.json').read().strip().splitlines()[-1]);print([round(v,4) for v in d['simulated']['rank_ms']], [round(v,4) for v in d['simulated']['rank_median_ms']])")" ;;
    kb:*)
      # per-kernel A/B (tools/kbench.py): kb:<job substrings, comma-separated>:<library builds, comma-separated>
      R=${S#kb:}; J=${R%%:*}; L=${R#*:}
      timeout -k 10 300 python tools/kbench.py --only "$J" --libs "$L" --reps 20 --rounds 3 > gpurun_out/${T}_kbench.txt 2>&1 || exit $?
      cat gpurun_out/${T}_kbench.txt | grep " med " ;;
    probe|probe:*|probegrads)
      E=${S#probe}; E=${E#:}; G=""; [ "$S" = probegrads ] && { E=""; G="--grads"; }
      env $E timeout -k 10 300 python tools/xagg_probe.py $G > gpurun_out/${T}_probe.txt 2>&1 || exit $?
      grep " us$" gpurun_out/${T}_probe.txt ;;
    simprof|simprof_ag|simprof_xa|simprof:*|simprof_ag:*|simprof_xa:*)
      # optional :<P> (default 8): rank 0 of the simulated P-rank step
      B=${S%%:*}; PP=8; [ "$B" != "$S" ] && PP=${S#*:}
      M=slab; [ "$B" = simprof_ag ] && M=allgather; [ "$B" = simprof_xa ] && M=xagg
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_${B}_P$PP -o run --output-format csv -- \
        python bench.py --simulate-world $PP --sim-rank 0 --dist-mode $M --steps 20 --warmup 3 > gpurun_out/${T}_${B}_P$PP.log 2>&1 || exit $?
      python tools/step_timeline.py gpurun_out/${T}_${B}_P$PP/run_kernel_trace.csv 10 > gpurun_out/${T}_${B}_P${PP}_timeline.txt || exit $?
      echo "$S ok" ;;
    align)
      # python -m hicgat.align (HiC_GAT_generalize_directly.py's flow) on GM12878 chr19 1 mb -> 500 kb,
      # 1000 fixed steps of the combined loss: (a) node2vec features made on the GPU (the reference's
      # configuration), (b) the alignment fixture's seeded embeddings x 0.1 (the GPU test's inputs)
      D=gpurun_out/${T}_align; mkdir -p $D
      python -c "
import numpy as np
a = np.load('tests/golden/align_chr19_f512.npz')
np.savetxt('$D/GM12878_1mb_chr19_list.txt', np.load('tests/golden/graph_chr19_1mb.npz')['list'], fmt='%d\t%d\t%.6f')
np.savetxt('$D/GM12878_500kb_chr19_list.txt', np.load('tests/golden/graph_chr19_500kb.npz')['list'], fmt='%d\t%d\t%.6f')
np.savetxt('$D/emb_1mb.txt', 0.1 * a['emb1'].astype(np.float64), fmt='%.9g')
np.savetxt('$D/emb_500kb.txt', 0.1 * a['emb2'].astype(np.float64), fmt='%.9g')" || exit 1
      (cd hic-gnn_amd && timeout -k 10 400 python -m hicgat.align ../$D/GM12878_1mb_chr19_list.txt ../$D/GM12878_500kb_chr19_list.txt \
        node2vec node2vec --steps 1000 --weights ../$D/n2v_weights.pt --out ../$D/n2v_GM12878_500kb_chr19 > ../$D/run_node2vec.log 2>&1) || exit $?
      (cd hic-gnn_amd && timeout -k 10 400 python -m hicgat.align ../$D/GM12878_1mb_chr19_list.txt ../$D/GM12878_500kb_chr19_list.txt \
        ../$D/emb_1mb.txt ../$D/emb_500kb.txt --steps 1000 --weights ../$D/fix_weights.pt --out ../$D/fix_GM12878_500kb_chr19 \
        > ../$D/run_fixture.log 2>&1) || exit $?
      tail -2 $D/run_node2vec.log $D/run_fixture.log ;;
    n2v)
      timeout -k 10 900 python tools/n2v_study.py gpurun_out/${T}_n2v_study.json > gpurun_out/${T}_n2v_study.log 2>&1; rc=$?
      tail -12 gpurun_out/${T}_n2v_study.log; [ $rc -eq 0 ] || exit $rc ;;
    n2vfix)
      timeout -k 10 300 python tests/golden/make_n2v_chr19.py gpurun_out/${T}_n2v_chr19_1mb_s43.npz 43 || exit $?
      timeout -k 10 300 python tests/golden/make_n2v_chr19.py gpurun_out/${T}_n2v_chr19_1mb_s42.npz 42 || exit $? ;;
    cli)
      mkdir -p gpurun_out/${T}_cli
      python -c "import numpy as np; d = np.load('tests/golden/graph_chr19_1mb.npz'); np.savetxt('gpurun_out/${T}_cli/GM12878_1mb_chr19_list.txt', d['list'], fmt='%d\t%d\t%.6f')" || exit 1
      (cd hic-gnn_amd && timeout -k 10 500 python -m hicgat.train ../gpurun_out/${T}_cli/GM12878_1mb_chr19_list.txt node2vec \
        --steps 1000 --out ../gpurun_out/${T}_cli/GM12878_1mb_chr19 > ../gpurun_out/${T}_cli/run.log 2>&1); rc=$?
      tail -5 gpurun_out/${T}_cli/run.log; [ $rc -eq 0 ] || exit $rc ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
echo "== all steps ok"
