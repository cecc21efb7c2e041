set -o pipefail
export TAG=d1
mkdir -p gpurun_out/$TAG
for c in ${CFGS:-4 3}; do
  timeout -k 10 180 python tools/diag_frame16_bar.py $c 8192 > gpurun_out/$TAG/bar_c$c.txt 2>&1 || { tail -5 gpurun_out/$TAG/bar_c$c.txt; exit 31; }
  grep -v amdgpu.ids gpurun_out/$TAG/bar_c$c.txt | head -60
done
[ -z "$NOSQ" ] && tools/gpu/run.sh sq:4
