# k_frame16 scheduler variants (make alt16 ALT_FLAGS=...): default vs
# -amdgpu-schedule-metric-bias=0 vs max-ilp, config 3, same box
set -o pipefail
export TAG=${TAG:-s8}
O=gpurun_out/$TAG
mkdir -p $O
for r in 1 2; do
  for v in def bias maxilp; do
    export TDOA_LIB=$PWD/audio-triangulation_amd/tdoa/libtdoa_f16_$v.so
    timeout -k 10 300 python bench.py --config 3 --no-cpu --no-parity > $O/c3_${v}_$r.json 2>$O/c3_${v}_$r.err || { tail -5 $O/c3_${v}_$r.err; exit 21; }
    tail -1 $O/c3_${v}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 $v r$r', '%.5g' % d['value'], '%.3f us' % (d['ms_per_step']*1e3), d.get('gpu_clock_mhz'))"
  done
done
