set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/round_end
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/round_end/tests.log 2>&1 &&
bash tools/measure_round.sh round_end
