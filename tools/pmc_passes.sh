#!/bin/bash
# PMC counter passes for the ray-march kernel (run on the GPU box via gpurun).
# One rocprofv3 run per counter group (--pmc with --kernel-trace only, no sys/runtime trace),
# each under its own time limit.  A counter-name error (exit 1) moves on to the next group;
# a timeout, abort, segfault or kill (124/134/137/139) stops everything.
# Usage: tools/pmc_passes.sh <tag> <counter-sets file> [tools/prof_run.py args...]
set -u
TAG=${1:-pmc}
SETS=${2:-tools/pmc_sets.txt}
shift 2 || true
ARGS=${*:-""}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -s KILL ${PASS_TIMEOUT:-90} rocprofv3 --kernel-trace --pmc $GROUP -d "$OUT/p$i" -o run --output-format csv \
      -- python3 tools/prof_run.py $ARGS > "$OUT/p$i.log" 2>&1 < /dev/null
  rc=$?
  echo "pass $i [$GROUP] rc=$rc" >> "$OUT/passes.txt"
  case $rc in
    124|134|137|139) echo "stopping after rc=$rc" >> "$OUT/passes.txt"; exit $rc ;;
  esac
done < "$SETS"
exit 0
