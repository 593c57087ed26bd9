# fused-loss kernel on the GPU box: kbench (full and math-only build) + the loss parity tests
set -o pipefail
mkdir -p gpurun_out
L=hic-gnn_amd/hicgat
timeout -k 10 300 python tools/kbench.py --only pairdist --reps 20 --libs $L/libhicgat.so,$L/libhicgat_d1.so > gpurun_out/kb_pd.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "fused_loss or pairdist or model_fixture or train_loop" -v --timeout 120 --timeout-method thread > gpurun_out/t_pd.log 2>&1; echo "tests rc=$?" >> gpurun_out/t_pd.log
echo done
