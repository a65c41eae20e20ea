set -o pipefail
O=gpurun_out/ws1; mkdir -p $O
timeout -k 10 300 python -m pytest tests -m gpu -q -x -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
for sh in 1 2 3; do
  for cfg in "--shading 0" "--shading 1 --ert 1e-5" "--dtype uint8 --n 256 --size 1024x1024"; do
    timeout -k 10 200 python tools/view_sweep.py $cfg --wave-shape $sh --reps 30 > $O/run.txt 2>&1 || exit $?
    python - "$sh" "$cfg" "$O/run.txt" <<'PY' | tee -a $O/ws.txt
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print("shape", sys.argv[1], sys.argv[2].ljust(40), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
  done
done
