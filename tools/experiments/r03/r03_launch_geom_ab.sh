#!/bin/bash
# Round 3: launch-geometry defines on the round-3 headline kernel: super-tile size
# (VR_SUPER_SHIFT 1/3 against 2), tile height (VR_MARCH_ROWS 8 against 16), re-ordering
# period of the adaptive tile order (VR_REORDER_EVERY 2/8 against 4), per-XCD list order
# (VR_LIST_ORDER 1 against 0).  C3 bench lines (K = 40), two alternating rounds.
set -o pipefail
TAG=${1:-r03_launch_geom}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
LIBSET=${LIBSET:-"lib lib_ss1 lib_ss3 lib_rows8 lib_re2 lib_re8 lib_lo1"}
for r in ${ROUNDS:-1 2}; do
  for L in $LIBSET; do
    VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 300 \
        python bench.py --config c3 --no-variants --no-cpu-baseline --steps 40 --warmup 10 \
        > $O/b_${L}_$r.json 2> $O/b_${L}_$r.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" \
        $O/b_${L}_$r.json $L | tee -a $O/summary.txt
  done
done
echo done > $O/rc.txt
