#!/bin/bash
# round-3 closing measurement, part 2: config 4 / config 5 lines (full-size parity) and rocprofv3
# kernel summaries of the headline and config-5 commands
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --model adaattn --steps 40 > gpurun_out/r03b_bench_aa4.json 2> gpurun_out/r03b_bench_aa4.err || exit 7
timeout -k 10 600 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 20 --prof-steps 3 --cpu-steps 1 --cpu-warmup 0 --no-vgg19 > gpurun_out/r03b_bench_aa5.json 2> gpurun_out/r03b_bench_aa5.err || exit 8
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03b_prof3 -o run -- \
  python3 bench.py --steps 20 --prof-steps 5 --no-cpu-baseline --no-vgg19 > gpurun_out/r03b_prof3.log 2>&1 || exit 9
python tools/prof_summary.py gpurun_out/r03b_prof3 30 > gpurun_out/r03b_kernel_summary.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03b_prof5 -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 5 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/r03b_prof5.log 2>&1 || exit 10
python tools/prof_summary.py gpurun_out/r03b_prof5 12 > gpurun_out/r03b_adaattn_c5_kernel_summary.txt 2>&1

echo done
