set -o pipefail
export TAG=f3
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh test smoke && \
tools/gpu/run.sh bench:3 bench:4 kstats:3 kstats:4
