#!/bin/bash
# PMC counter passes for the ray-march kernel (run on the GPU box via gpurun).
# One rocprofv3 run per counter group (--pmc with --kernel-trace only, no sys/runtime trace),
# each under its own time limit.  A counter-name error (exit 1) moves on to the next group;
# a timeout, abort, segfault or kill (124/134/137/139) stops everything.
# Usage: tools/pmc_passes.sh <tag> [bench args...]
set -u
TAG=${1:-pmc}
shift || true
ARGS=${*:-"--steps 10 --warmup 3 --no-cpu-baseline --no-variants"}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $GROUP -d "$OUT/p$i" -o run --output-format csv \
      -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i [$GROUP] rc=$rc" >> "$OUT/passes.txt"
  case $rc in
    124|134|137|139) echo "stopping after rc=$rc" >> "$OUT/passes.txt"; exit $rc ;;
  esac
done <<'EOF'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
TA_BUSY_avr TA_BUFFER_READ_WAVEFRONTS_sum TA_FLAT_READ_WAVEFRONTS_sum
SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS
GRBM_GUI_ACTIVE GRBM_COUNT
EOF
exit 0
