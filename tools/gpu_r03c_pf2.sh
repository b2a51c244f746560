#!/bin/bash
# PF2 (two stages of loads in flight, single-product GEMMs): bisect the train_video golden-step
# gradient error (conv only / wgrad only) and time config 5 with it off / on (A/B/A/B)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_r03b_pf2diag.sh || exit 3
for i in 1 2; do
  for pf in 0 1; do
    VST_PF2=$pf timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 3 --prof-steps 1 --no-cpu-baseline --no-vgg19 > gpurun_out/pf2_t${pf}_$i.json 2> gpurun_out/pf2_t${pf}_$i.err || exit 4
    python -c "import json;d=json.load(open('gpurun_out/pf2_t${pf}_$i.json'));print('PF2=$pf', d['ms_per_step'])"
  done
done
echo done
