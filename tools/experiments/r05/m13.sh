# build: the variants wrapped the field loads (field_rows_load) / the z-pair loads (zpair_load2) in __builtin_nontemporal_load under -DVR_FIELD_NT / -DVR_DENSITY_NT (lib_fnt / lib_dnt); removed after the A/B
# round 5: non-temporal (nt: L1-bypassing) loads for the binary16 field (lib_fnt) or for the
# density z-pairs (lib_dnt) against the default, alternating, 2 rounds; then L1/L2 counters
set -o pipefail
O=gpurun_out/r05_m13; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for b in lib lib_fnt lib_dnt; do
    for cfg in c3 c3_ref c3_default; do
      VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -k 10 150 python -u bench.py --config $cfg --no-variants --no-cpu-baseline --steps 40 --warmup 10 > $O/b_${b}_${cfg}_$r.json 2> $O/b_${b}_${cfg}_$r.err || exit 1
      python -c "import json,sys; d=json.load(open('$O/b_${b}_${cfg}_$r.json')); print('$b', '$cfg', $r, d['value'], d['ms_per_step'])"
    done
  done
done
for b in lib lib_fnt; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$b/libvr_amd.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TD_TD_BUSY_sum TD_TC_STALL_sum -d $O/pmc_${b} -o run --output-format csv -- python3 bench.py --config c3 --no-variants --no-cpu-baseline --steps 10 --warmup 3 > $O/pmc_${b}.log 2>&1 || exit 1
done
