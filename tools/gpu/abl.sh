# A/B two builds of libtdoa (tdoa/libtdoa.so vs tdoa/libtdoa_alt.so), interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in main alt; do
    if [ $v = alt ]; then export TDOA_LIB=$GRAFT_REPO_ROOT/audio-triangulation_amd/tdoa/libtdoa_alt.so; else unset TDOA_LIB; fi
    timeout -k 10 200 python bench.py --steps 400 --no-cpu > gpurun_out/abl_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/abl_$v.log; exit 21; }
    tail -1 gpurun_out/abl_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v r$r value %.4g kernel_ms %.4f' % (d['value'], d['roofline']['kernel_ms']))"
  done
done
