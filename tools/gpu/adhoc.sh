set -o pipefail
export TAG=p3s
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh test:tests/test_gpu_bench_path.py,tests/test_gpu_frame16_variants.py,tests/test_ls.py,tests/test_gpu_gcc_phat.py && \
STEPS=5 BENCH_ARGS="--config 4 --no-parity --no-cpu" tools/gpu/run.sh ablib:libtdoa,libtdoa_p3s0,libtdoa,libtdoa_p3s0 && \
STEPS=20 BENCH_ARGS="--config 3 --no-parity --no-cpu" tools/gpu/run.sh ablib:libtdoa,libtdoa_p3s0,libtdoa,libtdoa_p3s0
