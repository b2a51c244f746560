#!/bin/bash
# channel_dot float4 form (unrolled) vs the scalar form on config 5 (A/B/A/B, VST_CDOT_VEC) + unit tests
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_elementwise.py tests/test_gpu_adaattn.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/cdot_tests.log 2>&1 || { tail -40 gpurun_out/cdot_tests.log; exit 4; }
tail -2 gpurun_out/cdot_tests.log
for i in 1 2; do
  for v in 0 1; do
    VST_CDOT_VEC=$v timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 3 --prof-steps 1 --no-cpu-baseline --no-vgg19 > gpurun_out/cdot${v}_$i.json 2>/dev/null || exit 5
    python -c "import json;d=json.load(open('gpurun_out/cdot${v}_$i.json'));print('c5 cdot_vec=$v', round(d['ms_per_step'],2))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cdot_prof -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 3 --prof-steps 1 --no-cpu-baseline --no-vgg19 > gpurun_out/cdot_prof.log 2>&1 || exit 6
grep -h channel_dot gpurun_out/cdot_prof/run_kernel_stats.csv
echo done
