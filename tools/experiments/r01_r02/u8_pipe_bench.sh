O=gpurun_out/r02_u8b; mkdir -p $O
for L in lib lib_quad; do for pp in 0 1; do for cfg in c2 c4; do
  VR_PIPELINE=$pp VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 300 python bench.py --config $cfg --no-variants --no-cpu-baseline --steps 30 > $O/b.json 2> $O/b.err || exit 1
  python -c "import json; d=json.load(open('$O/b.json')); print('$L', 'pipe=$pp', '$cfg', d['value'], d['ms_per_step'])" | tee -a $O/out.txt
done; done; done
