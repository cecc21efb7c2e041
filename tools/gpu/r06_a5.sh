set -o pipefail
export TAG=a5
mkdir -p gpurun_out/$TAG
for l in ${LIBS:-libtdoa_dump0 libtdoa_dump1}; do
  for c in 3 4; do
    TDOA_LIB=$GRAFT_REPO_ROOT/audio-triangulation_amd/tdoa/$l.so timeout -k 10 120 python tools/diag_rng.py $c > gpurun_out/$TAG/rng_${l}_$c.txt 2>&1
    echo "$l c$c rc=$?"; tail -14 gpurun_out/$TAG/rng_${l}_$c.txt
  done
done
