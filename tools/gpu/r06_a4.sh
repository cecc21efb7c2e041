set -o pipefail
export TAG=a4
mkdir -p gpurun_out/$TAG
for l in libtdoa_rngs2 libtdoa_rngs; do
  TDOA_LIB=$GRAFT_REPO_ROOT/audio-triangulation_amd/tdoa/$l.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_path.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/pytest_$l.log 2>&1
  echo "$l rc=$?"; grep -E "passed|failed|Error:" gpurun_out/$TAG/pytest_$l.log | tail -4
done
