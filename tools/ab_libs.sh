#!/bin/bash
# A/B timing of alternate libtdoa builds (tools only): each library runs the
# default bench line (config 2 unless ARGS says otherwise) ROUNDS times, in
# interleaved order, printing kernel us and loc/s per run.
#   tools/ab_libs.sh "base asmmul unit" [ROUNDS] [ARGS...]
cd "$(dirname "$0")/.."
names=$1; rounds=${2:-2}; shift 2 || shift $#
for r in $(seq 1 "$rounds"); do
  for n in $names; do
    lib=audio-triangulation_amd/tdoa/libtdoa_x_$n.so
    out=$(TDOA_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu --no-parity "$@" 2>/dev/null | tail -1)
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print(f'{sys.argv[1]:10s} kernel {d[\"roofline\"][\"kernel_ms\"]*1e3:7.2f} us  {d[\"value\"]:.4g} loc/s')" "$n" "$out" || exit 1
  done
done
