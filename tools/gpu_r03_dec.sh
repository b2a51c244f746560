#!/bin/bash
# decoder ReLU-mask fusion (correctness: unit chain + AdaAttN step tests) and the 256x256
# single-product conv tile A/B (VST_T256W) on the config-5 step, one box
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_adaattn.py -q -x --timeout 300 --timeout-method thread \
  -k "masked_dgrad or train_video or midsize or decoder or units_golden" > gpurun_out/r03_dec_tests.log 2>&1 || exit 3
for i in 1 2; do
for w in 0 1; do
  VST_T256W=$w timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/r03_t256w_${w}_$i.json 2>gpurun_out/r03_t256w_${w}_$i.err || exit 5
done; done
VST_T256W=1 timeout -k 10 600 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 5 --prof-steps 2 --cpu-steps 1 --cpu-warmup 0 --no-vgg19 > gpurun_out/r03_t256w_par.json 2>gpurun_out/r03_t256w_par.err || exit 6
echo done
