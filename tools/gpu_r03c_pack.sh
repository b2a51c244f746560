#!/bin/bash
# pack_matrix row form: elementwise + AdaAttN GPU tests, config-5 step timing and its kernel profile
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_elementwise.py tests/test_gpu_adaattn.py tests/test_gpu_abi.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pack_tests.log 2>&1 || { tail -40 gpurun_out/pack_tests.log; exit 4; }
tail -2 gpurun_out/pack_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 3 --prof-steps 1 --no-cpu-baseline --no-vgg19 > gpurun_out/pack_c5_$i.json 2>/dev/null || exit 5
  python tools/show_bench.py gpurun_out/pack_c5_$i.json | head -1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pack_prof -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 5 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/pack_prof.log 2>&1 || exit 6
python tools/prof_summary.py gpurun_out/pack_prof 12 > gpurun_out/pack_c5_kernel_summary.txt 2>&1
grep -h pack_matrix gpurun_out/pack_prof/run_kernel_stats.csv
echo done
