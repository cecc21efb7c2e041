# k_frame16 frames from a queue (F16_DYN; libtdoa_dyn0 = the static stride)
set -o pipefail
export TAG=${TAG:-q3}
O=gpurun_out/$TAG
mkdir -p $O
L=$GRAFT_REPO_ROOT/audio-triangulation_amd/tdoa
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_path.py tests/test_gpu_gcc_phat.py tests/test_gpu_bench_sizes.py tests/test_gpu_frame16_variants.py -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 20; }
tail -1 $O/pytest.log
for c in 4 3; do
  for r in 1 2; do
    for l in libtdoa_dyn0 libtdoa; do
      TDOA_LIB=$L/$l.so timeout -k 10 240 python bench.py --config $c --no-cpu --no-parity > $O/ab_c${c}_${l}_$r.json 2>$O/ab_c${c}_${l}_$r.err || { echo "bench $c $l failed"; tail -5 $O/ab_c${c}_${l}_$r.err; exit 21; }
      tail -1 $O/ab_c${c}_${l}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c$c $l r$r', '%.5g' % d['value'], '%.3f ms' % d['ms_per_step'], d.get('gpu_clock_mhz'))"
    done
  done
done
timeout -k 10 180 python tools/diag_frame16_bar.py 4 8192 > $O/bar_c4.txt 2>&1 || { tail -5 $O/bar_c4.txt; exit 31; }
grep "stamped frame" $O/bar_c4.txt
