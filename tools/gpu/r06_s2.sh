# config 5: batched staging loads in k_direct_mfma<.., EMA> (same-box A/B
# against the previous build, libtdoa_base.so) + parity + phase split
set -o pipefail
export TAG=${TAG:-s2}
O=gpurun_out/$TAG
mkdir -p $O
L=$GRAFT_REPO_ROOT/audio-triangulation_amd/tdoa
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_bench_sizes.py -k "stream or c5 or config5" -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 20; }
tail -1 $O/pytest.log
for r in 1 2; do
  for l in libtdoa_base libtdoa; do
    TDOA_LIB=$L/$l.so timeout -k 10 300 python bench.py --config 5 --engine direct --no-cpu --no-parity > $O/c5_${l}_$r.json 2>$O/c5_${l}_$r.err || { tail -5 $O/c5_${l}_$r.err; exit 21; }
    tail -1 $O/c5_${l}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$l r$r', '%.5g' % d['value'], '%.2f us' % (d['ms_per_step']*1e3), d.get('gpu_clock_mhz'))"
  done
done
timeout -k 10 180 python tools/diag_stream_phases.py > $O/phases.txt 2>&1 || { tail -5 $O/phases.txt; exit 31; }
grep -v amdgpu.ids $O/phases.txt | head -9
