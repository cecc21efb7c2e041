set -o pipefail
export TAG=m2
tools/gpu/run.sh test:tests/test_gpu_frame16_variants.py,tests/test_gpu_bench_path.py && \
STEPS=5 ROUNDS=1 BENCH_ARGS="--config 4 --no-parity" tools/gpu/run.sh abenv:TDOA_F16_FG:1,0,skip && \
STEPS=20 ROUNDS=1 BENCH_ARGS="--config 3 --no-parity" tools/gpu/run.sh abenv:TDOA_F16_FG:1,0,skip && \
STEPS=50 tools/gpu/run.sh kstats:5 && \
tools/gpu/run.sh flops:2 && \
BENCH_ARGS="--batch 65536" tools/gpu/run.sh flops:3 && \
BENCH_ARGS="--batch 131072" tools/gpu/run.sh flops:4 && \
tools/gpu/run.sh calib
