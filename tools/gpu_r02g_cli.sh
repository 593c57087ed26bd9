#!/bin/bash
# round-2 closing: the reference driver's flow on GM12878 chr19 1 mb (configs[0]) through the CLI,
# node2vec features generated on the GPU, the reference's default conversion sweep [.1,.1,2], fixed
# 1000 steps per conversion (bounded run time); log, structure and weights under gpurun_out/cli/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cli
export TMPDIR=/tmp
python - <<'PY' || exit 1
import numpy as np
d = np.load("tests/golden/graph_chr19_1mb.npz")
np.savetxt("gpurun_out/cli/GM12878_1mb_chr19_list.txt", d["list"], fmt="%d\t%d\t%.6f")
PY
cd hic-gnn_amd
timeout -k 10 500 python -m hicgat.train ../gpurun_out/cli/GM12878_1mb_chr19_list.txt node2vec --steps 1000 --out ../gpurun_out/cli/GM12878_1mb_chr19 > ../gpurun_out/cli/run.log 2>&1; rc=$?
tail -25 ../gpurun_out/cli/run.log
exit $rc
