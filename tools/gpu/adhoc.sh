set -o pipefail
export TAG=m6
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh bench:3 bench:4 bench:2 bench:5:direct && \
tools/gpu/run.sh kstats:3 kstats:4 pmc:3 pmc:4
