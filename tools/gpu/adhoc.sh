set -o pipefail
export TAG=L2
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh test:tests/test_gpu_gcc_phat.py,tests/test_gpu_bench_path.py,tests/test_gpu_frame16_variants.py,tests/test_ls.py && \
STEPS=8 BENCH_ARGS="--config 4" tools/gpu/run.sh ablib:libtdoa_L1,libtdoa,libtdoa_L1,libtdoa,libtdoa_L1,libtdoa && \
STEPS=60 BENCH_ARGS="--config 3" tools/gpu/run.sh ablib:libtdoa_L1,libtdoa
