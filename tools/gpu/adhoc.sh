set -o pipefail
export TAG=c3d
mkdir -p gpurun_out/$TAG
STEPS=20 ROUNDS=2 BENCH_ARGS="--config 3" tools/gpu/run.sh abenv:TDOA_F16_DEFER:0,1
