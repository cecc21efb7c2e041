set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python tools/diag_p1k.py 4096 > gpurun_out/p1k_diag.txt 2>&1; cat gpurun_out/p1k_diag.txt | tail -16
