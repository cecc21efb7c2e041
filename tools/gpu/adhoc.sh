set -o pipefail
export TAG=s1
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh test:tests/test_gpu_stream.py,tests/test_gpu_parity.py,tests/test_gpu_variants.py && \
STEPS=400 BENCH_ARGS="--config 5 --engine direct" tools/gpu/run.sh ablib:libtdoa_e0,libtdoa_eA,libtdoa,libtdoa_e0,libtdoa_eA,libtdoa,libtdoa_e0,libtdoa_eA,libtdoa
