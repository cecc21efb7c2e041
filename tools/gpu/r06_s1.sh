# config 5: what the streaming EMA launch's empty workgroups cost
# (TDOA_DIRECT_RESGRID, A/B library only) and the per-phase split
set -o pipefail
export TAG=${TAG:-s1}
O=gpurun_out/$TAG
mkdir -p $O
L=$GRAFT_REPO_ROOT/audio-triangulation_amd/tdoa
TDOA_LIB=$L/libtdoa_ab.so TDOA_DIRECT_RESGRID=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_resgrid.log 2>&1 || { tail -20 $O/pytest_resgrid.log; exit 20; }
tail -1 $O/pytest_resgrid.log
for r in 1 2; do
  for v in 0 1; do
    TDOA_LIB=$L/libtdoa_ab.so TDOA_DIRECT_RESGRID=$v timeout -k 10 300 python bench.py --config 5 --engine direct --no-cpu --no-parity > $O/c5_rg${v}_$r.json 2>$O/c5_rg${v}_$r.err || { tail -5 $O/c5_rg${v}_$r.err; exit 21; }
    tail -1 $O/c5_rg${v}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('resgrid=$v r$r', '%.5g' % d['value'], '%.2f us' % (d['ms_per_step']*1e3), d.get('gpu_clock_mhz'))"
  done
done
for v in 0 1; do
  TDOA_DIRECT_RESGRID=$v timeout -k 10 180 python tools/diag_stream_phases.py > $O/phases_rg$v.txt 2>&1 || { tail -5 $O/phases_rg$v.txt; exit 31; }
  grep -v amdgpu.ids $O/phases_rg$v.txt | tail -12
done
