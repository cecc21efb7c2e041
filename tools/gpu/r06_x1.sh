# k_direct_mfma three-mic xcorr units (kp.xc3: (frame, first mic) tiles, two per
# frame instead of three): parity, same-box A/B (TDOA_DIRECT_XC3=0 / 1) at
# config 5 and config 2 DIRECT, phase split
set -o pipefail
export TAG=${TAG:-x1}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_parity.py tests/test_gpu_variants.py tests/test_gpu_bench_sizes.py -k "not long_frames" -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 20; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in 0 1; do
    TDOA_DIRECT_XC3=$v timeout -k 10 300 python bench.py --config 5 --engine direct --no-cpu --no-parity > $O/c5_x${v}_$r.json 2>$O/c5_x${v}_$r.err || { tail -5 $O/c5_x${v}_$r.err; exit 21; }
    tail -1 $O/c5_x${v}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 xc3=$v r$r', '%.5g' % d['value'], '%.2f us' % (d['ms_per_step']*1e3), d.get('gpu_clock_mhz'))"
    TDOA_DIRECT_XC3=$v timeout -k 10 300 python bench.py --config 2 --engine direct --no-cpu --no-parity > $O/c2d_x${v}_$r.json 2>$O/c2d_x${v}_$r.err || { tail -5 $O/c2d_x${v}_$r.err; exit 22; }
    tail -1 $O/c2d_x${v}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 direct xc3=$v r$r', '%.5g' % d['value'], '%.2f us' % (d['ms_per_step']*1e3), d.get('gpu_clock_mhz'))"
  done
done
for v in 0 1; do
  TDOA_DIRECT_XC3=$v timeout -k 10 180 python tools/diag_stream_phases.py > $O/phases_x$v.txt 2>&1 || { tail -5 $O/phases_x$v.txt; exit 31; }
  grep -v amdgpu.ids $O/phases_x$v.txt | head -8
done
