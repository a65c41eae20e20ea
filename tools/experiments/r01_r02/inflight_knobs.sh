O=gpurun_out/r02_inflight_knobs; mkdir -p $O
for v in default diag fill; do for arm in "base:" "pair2:VR_PAIR=1" "pair4:VR_PAIR=1 VR_PAIR_LANES=4"; do
  name=${arm%%:*}; envs=${arm#*:}
  for sh in "--shading 1 --ert 1e-5" "--shading 0 --ert 0"; do
  echo "== $v $name $sh" >> $O/out.txt
  env $envs timeout -k 10 120 python tools/inflight_sweep.py --view $v --ranks 1 --streams 3 --frames 150 $sh >> $O/out.txt 2>> $O/err.txt || exit 1
  done
done; done
