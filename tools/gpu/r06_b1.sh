set -o pipefail
export TAG=b1
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh test:tests/test_gpu_bench_sizes.py,tests/test_gpu_bench_path.py,tests/test_ls.py && \
STEPS=5 ROUNDS=2 BENCH_ARGS="--config 4" tools/gpu/run.sh abenv:TDOA_F16_CHUNK:0,16384,32768 && \
BENCH_ARGS="" tools/gpu/run.sh pmc:4 && \
TDOA_F16_CHUNK=0 TAG=b1n tools/gpu/run.sh pmc:4
