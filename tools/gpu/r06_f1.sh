set -o pipefail
export TAG=${TAG:-f1}
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh test smoke && \
tools/gpu/run.sh bench:2 && \
BENCH_ARGS="--steps 20 --warmup 5" TAG=${TAG}d tools/gpu/run.sh bench:2 && \
tools/gpu/run.sh bench:2:direct bench:3 bench:4 bench:5:direct bench:1:direct && \
tools/gpu/run.sh kstats:2 kstats:3 kstats:4 kstats:5:direct
