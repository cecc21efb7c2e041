# k_p1k_lean scheduler variants (make alt ALT_FLAGS=...): default vs
# -amdgpu-schedule-metric-bias=0, same box, config 2 (400 steps)
set -o pipefail
export TAG=${TAG:-s7}
O=gpurun_out/$TAG
mkdir -p $O
for r in 1 2 3; do
  for v in def bias; do
    export TDOA_LIB=$PWD/audio-triangulation_amd/tdoa/libtdoa_p1k_$v.so
    timeout -k 10 300 python bench.py --config 2 --no-cpu --no-parity > $O/c2_${v}_$r.json 2>$O/c2_${v}_$r.err || { tail -5 $O/c2_${v}_$r.err; exit 21; }
    tail -1 $O/c2_${v}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 $v r$r', '%.5g' % d['value'], '%.3f us' % (d['ms_per_step']*1e3), d.get('gpu_clock_mhz'))"
  done
done
