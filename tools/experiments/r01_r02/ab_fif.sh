# N=1 C3: frames in flight 2 vs 3 vs 4 (stable tile order)
set -o pipefail
O=gpurun_out/ab_fif; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do for F in 3 2 4; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-variants --frames-in-flight $F > $O/bench_f${F}_$r.json 2> $O/bench_f${F}_$r.err || exit $?
done; done
