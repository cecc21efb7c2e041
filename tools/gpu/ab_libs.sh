# A/B of the config-2 bench across library variants (tdoa/libtdoa_alt_*.so) vs the default build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/ab
run() {
  n=$1; lib=$2
  TDOA_LIB=$lib timeout -k 10 200 python bench.py --steps 400 --no-cpu > gpurun_out/ab/$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/ab/$n.log; return 1; }
  tail -1 gpurun_out/ab/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n value %.4g kernel_ms %.5f' % (d['value'], d['roofline']['kernel_ms']))"
}
run base audio-triangulation_amd/tdoa/libtdoa.so || exit 1
for f in audio-triangulation_amd/tdoa/libtdoa_alt_*.so; do
  n=$(basename $f .so); run $n $f || exit 1
done
run base2 audio-triangulation_amd/tdoa/libtdoa.so
