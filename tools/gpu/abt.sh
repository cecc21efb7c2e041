# A/B two builds (tdoa/libtdoa.so vs tdoa/libtdoa_alt.so): GCC-PHAT parity tests on
# the alt build, then interleaved bench runs of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TDOA_LIB=$GRAFT_REPO_ROOT/audio-triangulation_amd/tdoa/libtdoa_alt.so timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_gcc_phat.py} -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/abt_test.log 2>&1
rc=$?; echo "alt tests rc=$rc"; tail -4 gpurun_out/abt_test.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/abl.sh
