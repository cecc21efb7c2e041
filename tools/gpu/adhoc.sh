set -o pipefail
export TAG=full6
mkdir -p gpurun_out/$TAG
tools/gpu/run.sh test smoke
