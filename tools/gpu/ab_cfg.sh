# A/B of bench configs (CFGS, default "5 2d") across library variants (tdoa/libtdoa_alt_*.so) vs the default build.
# "2d" = config 2 on the DIRECT engine.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/ab
run() {
  n=$1; lib=$2; shift 2
  TDOA_LIB=$lib timeout -k 10 200 python bench.py --no-cpu "$@" > gpurun_out/ab/$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/ab/$n.log; return 1; }
  tail -1 gpurun_out/ab/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n $* value %.4g ms %.5f' % (d['value'], d['ms_per_step']))"
}
for f in audio-triangulation_amd/tdoa/libtdoa.so audio-triangulation_amd/tdoa/libtdoa_alt_*.so; do
  n=$(basename $f .so)
  for c in ${CFGS:-5 2d}; do
    if [ "$c" = "2d" ]; then run $n $f --engine direct --steps 200 || exit 1
    else run $n $f --config $c || exit 1; fi
  done
done
