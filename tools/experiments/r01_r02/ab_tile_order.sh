set -o pipefail
O=gpurun_out/to1; mkdir -p $O
for rep in 1 2; do
for to in 3 4; do
  for cfg in "--shading 1 --ert 1e-5" "--shading 0" "--shading 1 --ert 1e-5 --skip-empty 1"; do
    timeout -k 10 200 python tools/view_sweep.py $cfg --tile-order $to --reps 30 > $O/run.txt 2>&1 || exit $?
    python - "$to" "$cfg" "$O/run.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print("order", sys.argv[1], sys.argv[2].ljust(40), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
  done
done
done
