set -o pipefail
export TAG=noout
mkdir -p gpurun_out/$TAG
STEPS=5 BENCH_ARGS="--config 4 --no-parity --no-cpu" tools/gpu/run.sh ablib:libtdoa,libtdoa_noout,libtdoa,libtdoa_noout && \
STEPS=20 BENCH_ARGS="--config 3 --no-parity --no-cpu" tools/gpu/run.sh ablib:libtdoa,libtdoa_noout,libtdoa,libtdoa_noout
