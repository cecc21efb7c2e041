set -o pipefail
export TAG=lag3
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh test:tests/test_gpu_bench_path.py,tests/test_gpu_frame16_variants.py,tests/test_ls.py && \
for l in libtdoa libtdoa_lag0 libtdoa libtdoa_lag0; do
  TDOA_LIB=$PWD/audio-triangulation_amd/tdoa/$l.so timeout -k 10 120 python tools/time_launch.py 4 131072 10 || exit 5
done && \
STEPS=5 BENCH_ARGS="--config 4 --no-parity --no-cpu" tools/gpu/run.sh ablib:libtdoa,libtdoa_lag0,libtdoa,libtdoa_lag0
