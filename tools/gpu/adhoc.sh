set -o pipefail
export TAG=f2
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh test smoke && \
tools/gpu/run.sh bench:2 bench:3 bench:4 && \
tools/gpu/run.sh kstats:3 kstats:4
