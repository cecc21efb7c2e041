set -o pipefail
export TAG=t2
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh test:tests/test_gpu_gcc_phat.py,tests/test_gpu_bench_path.py && \
STEPS=400 tools/gpu/run.sh ablib:libtdoa_tw0,libtdoa_tw7,libtdoa,libtdoa_tw0,libtdoa_tw7,libtdoa,libtdoa_tw0,libtdoa_tw7,libtdoa && \
tools/gpu/run.sh pmc:2
