# config 5 pipelined hops: trigger stream priority A/B, plus the two-pipeline bound
set -o pipefail
export TAG=${TAG:-q2}
O=gpurun_out/$TAG
mkdir -p $O
for r in 1 2; do
  for m in "stream 1" "pipelined 1" "pipelined 0"; do
    set -- $m
    TDOA_STREAM_PIPE_PRIO=$2 timeout -k 10 300 python bench.py --config 5 --engine direct --stream-mode $1 --no-cpu --no-parity > $O/c5_$1$2_$r.json 2>$O/c5_$1$2_$r.err || { tail -5 $O/c5_$1$2_$r.err; exit 21; }
    tail -1 $O/c5_$1$2_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 $1 prio=$2 r$r', '%.5g' % d['value'], '%.2f us' % (d['ms_per_step']*1e3), 'lat p50 %.4f' % d['latency_ms']['p50'], d.get('gpu_clock_mhz'))"
  done
done
