# DIRECT grid solve: unguarded slot reads (non-streaming kernel), same-box A/B
# against libtdoa_gbase.so (the guarded form) + DIRECT parity
set -o pipefail
export TAG=${TAG:-g1}
O=gpurun_out/$TAG
mkdir -p $O
L=$GRAFT_REPO_ROOT/audio-triangulation_amd/tdoa
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_variants.py tests/test_gpu_stream.py -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 20; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for l in libtdoa_gbase libtdoa; do
    TDOA_LIB=$L/$l.so timeout -k 10 300 python bench.py --config 2 --engine direct --no-cpu --no-parity > $O/c2d_${l}_$r.json 2>$O/c2d_${l}_$r.err || { tail -5 $O/c2d_${l}_$r.err; exit 21; }
    tail -1 $O/c2d_${l}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 direct $l r$r', '%.5g' % d['value'], '%.2f us' % (d['ms_per_step']*1e3), d.get('gpu_clock_mhz'))"
  done
done
