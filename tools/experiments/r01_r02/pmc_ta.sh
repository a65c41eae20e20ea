# gather-pipeline counters (TA / TD / TCP / SQ, one rocprofv3 pass per group) for C3 and the
# reference-semantics frame
set -o pipefail
bash tools/pmc_passes.sh pmc_ta_c3 tools/pmc_sets_ta.txt --shading 1 --ert 1e-5 --frames 10 &&
bash tools/pmc_passes.sh pmc_ta_ref tools/pmc_sets_ta.txt --shading 0 --ert 0 --frames 10
