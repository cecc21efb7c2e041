set -o pipefail
export TAG=m7
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh test smoke && \
tools/gpu/run.sh bench:3 bench:4 && \
tools/gpu/run.sh kstats:3 kstats:4 pmc:3 pmc:4
