#!/bin/bash
# round-2 benches: headline (bf16x6, default), f32 policy, AdaAttN config-4 / config-5 shapes,
# then rocprofv3 kernel stats of the headline and of config 5
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/r02_bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gemm f32 --steps 60 > gpurun_out/r02_bench_f32.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model adaattn --steps 40 --no-cpu-baseline > gpurun_out/r02_bench_aa4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 2 --no-cpu-baseline --no-vgg19 > gpurun_out/r02_bench_aa5.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02_prof_rc -o run -- \
  python3 bench.py --steps 20 --prof-steps 5 --no-cpu-baseline --no-vgg19 > gpurun_out/r02_prof_rc.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02_prof_aa5 -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 4 --warmup 1 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/r02_prof_aa5.log 2>&1 || exit $?
echo done
