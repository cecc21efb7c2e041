# k_frame16 issue-priority A/B (F16_PRIO, libtdoa_prio1/2 from `make alt16`)
# and the barrier-wait split with the fixed diagnostic library
set -o pipefail
export TAG=${TAG:-p1}
O=gpurun_out/$TAG
mkdir -p $O
L=$GRAFT_REPO_ROOT/audio-triangulation_amd/tdoa
for c in 4 3; do
  timeout -k 10 180 python tools/diag_frame16_bar.py $c 8192 > $O/bar_c$c.txt 2>&1 || { tail -5 $O/bar_c$c.txt; exit 31; }
  TDOA_LIB=$L/libtdoa_diag_prio1.so timeout -k 10 180 python tools/diag_frame16_bar.py $c 8192 > $O/bar_prio1_c$c.txt 2>&1 || { tail -5 $O/bar_prio1_c$c.txt; exit 32; }
  grep "stamped frame" $O/bar_c$c.txt $O/bar_prio1_c$c.txt
done
for c in 4 3; do
  for r in 1 2; do
    for l in libtdoa libtdoa_prio1 libtdoa_prio2; do
      TDOA_LIB=$L/$l.so timeout -k 10 240 python bench.py --config $c --no-cpu --no-parity > $O/ab_c${c}_${l}_$r.json 2>$O/ab_c${c}_${l}_$r.err || { echo "bench $c $l failed"; tail -5 $O/ab_c${c}_${l}_$r.err; exit 21; }
      tail -1 $O/ab_c${c}_${l}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c$c $l r$r', '%.5g' % d['value'], '%.3f ms' % d['ms_per_step'], d.get('gpu_clock_mhz'))"
    done
  done
done
