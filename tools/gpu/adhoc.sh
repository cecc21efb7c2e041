set -o pipefail
export TAG=sub
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh test:tests/test_gpu_gcc_phat.py,tests/test_gpu_parity.py,tests/test_gpu_bench_path.py && \
STEPS=400 tools/gpu/run.sh ablib:libtdoa,libtdoa_subor,libtdoa,libtdoa_subor,libtdoa,libtdoa_subor
