# round 5: frames in flight 3 (default) / 4 / 6 on the shipped build, alternating, 2 rounds
set -o pipefail
O=gpurun_out/r05_m16; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for f in 3 4 6 2; do
    for cfg in c3 c3_ref c3_default; do
      timeout -k 10 150 python -u bench.py --config $cfg --frames-in-flight $f --no-variants --no-cpu-baseline --steps 40 --warmup 10 > $O/b_${f}_${cfg}_$r.json 2> $O/b_${f}_${cfg}_$r.err || exit 1
      python -c "import json,sys; d=json.load(open('$O/b_${f}_${cfg}_$r.json')); print('fif=$f', '$cfg', $r, d['value'], d['ms_per_step'])"
    done
  done
done
