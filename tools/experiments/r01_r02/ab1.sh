set -o pipefail
O=gpurun_out/ab1; mkdir -p $O
R="timeout -k 10 120 python tools/prof_run.py --frames 30"
$R --shading 1 > $O/shaded_pipe.json &&
VR_PIPELINE=0 $R --shading 1 > $O/shaded_nopipe.json &&
$R --shading 0 > $O/unshaded_ert.json &&
VR_PIPELINE=1 $R --shading 0 > $O/unshaded_ert_pipe.json &&
$R --shading 0 --ert 0 > $O/ref.json &&
VR_PIPELINE=1 $R --shading 0 --ert 0 > $O/ref_pipe.json
