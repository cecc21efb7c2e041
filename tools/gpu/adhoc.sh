set -o pipefail
export TAG=d5
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh diagf16:4 && \
timeout -k 10 120 python tools/diag_grid_bb.py 4 262144 > gpurun_out/$TAG/diag_bb_c4.txt 2>&1 && cat gpurun_out/$TAG/diag_bb_c4.txt && \
tools/gpu/run.sh test:tests/test_gpu_frame16_variants.py
