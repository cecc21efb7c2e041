set -o pipefail
export TAG=f1
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh test smoke && \
tools/gpu/run.sh bench:2 bench:3 bench:4 bench:5:direct bench:2:direct bench:1 && \
tools/gpu/run.sh kstats:2 kstats:3 kstats:4 kstats:5:direct
