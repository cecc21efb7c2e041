set -o pipefail
export TAG=t1
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh test:tests/test_gpu_gcc_phat.py,tests/test_gpu_bench_path.py,tests/test_gpu_parity.py && \
STEPS=400 tools/gpu/run.sh ablib:libtdoa_tw0,libtdoa,libtdoa_tw0,libtdoa,libtdoa_tw0,libtdoa
