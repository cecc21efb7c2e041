set -o pipefail
export TAG=a2
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh test testlib:libtdoa_rngs:tests/test_gpu_bench_path.py smoke bench:2
