set -o pipefail
export TAG=n1
mkdir -p gpurun_out/$TAG
STEPS=8 BENCH_ARGS="--config 4" tools/gpu/run.sh ablib:libtdoa_nolag,libtdoa,libtdoa_nolag,libtdoa && \
STEPS=60 BENCH_ARGS="--config 3" tools/gpu/run.sh ablib:libtdoa_nolag,libtdoa,libtdoa_nolag,libtdoa
