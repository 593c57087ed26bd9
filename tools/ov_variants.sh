set -e
b() { timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@"; }
b > gpurun_out/v_g_ov.log 2>&1
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 b > gpurun_out/v_gpc0_ov.log 2>&1
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 HICGAT_OVERLAP=0 b > gpurun_out/v_gpc0_noov.log 2>&1
b --eager > gpurun_out/v_e_ov.log 2>&1
HICGAT_OVERLAP=0 b --eager > gpurun_out/v_e_noov.log 2>&1
