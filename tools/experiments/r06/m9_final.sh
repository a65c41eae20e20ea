#!/bin/bash
# round 6 final measurement: tools/measure_round.sh for every config (smoke, bench_noV, rocprof
# kernel-trace summary, FETCH_SIZE/WRITE_SIZE passes -> profiles/pmc_traffic.json, bench.json)
cd "$GRAFT_REPO_ROOT"
bash tools/measure_round.sh r06_final "c3 c3_default c3_ref c2 c4 c5"
