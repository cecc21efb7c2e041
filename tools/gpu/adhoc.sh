set -o pipefail
export TAG=m8
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh test smoke && \
tools/gpu/run.sh bench:3 bench:4 && \
tools/gpu/run.sh kstats:3 kstats:4 pmc:3 pmc:4 && \
timeout -k 10 120 python tools/diag_grid_bb.py 4 262144 > gpurun_out/$TAG/diag_bb_c4.txt 2>&1 && cat gpurun_out/$TAG/diag_bb_c4.txt
