#!/bin/bash
# A/B of two k-tiles per stage in the single-product conv GEMMs (VST_KD2) on the config-5 step, the
# AdaAttN GPU tests, and a rocprofv3 kernel summary of the default build
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_adaattn.py tests/test_abi.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/kd_tests.log 2>&1 || exit 2
i=0
for kd in 0 1 0 1; do
  i=$((i+1))
  VST_KD2=$kd timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 3 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/kd_aa5_${kd}_$i.json 2> gpurun_out/kd_aa5_$i.err || exit 5
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kd_prof -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 5 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/kd_prof.log 2>&1 || exit 6
python tools/prof_summary.py gpurun_out/kd_prof 10 -shapes > gpurun_out/kd_summary.txt 2>&1
echo done
