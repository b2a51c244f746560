#!/bin/bash
# closing measurement of a round's final build (usage: tools/gpu_close.sh r06): GPU suite + smoke(), the headline line as the driver
# runs it (defaults), the strict-f32 line, config-4 and config-5 lines (full-size parity), and the
# rocprofv3 kernel summaries of the headline and config-5 steps (side streams off, as bench.py's
# instrumented steps, so the per-kernel averages compare)
cd $GRAFT_REPO_ROOT
R=${1:-r06}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_tests.log 2>&1 || { tail -40 gpurun_out/${R}_tests.log; exit 4; }
tail -2 gpurun_out/${R}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 5
timeout -k 10 600 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit 6
python tools/show_bench.py gpurun_out/${R}_bench.json | head -2
timeout -k 10 300 python bench.py --gemm f32 --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/${R}_bench_f32.json 2>/dev/null || exit 7
python tools/show_bench.py gpurun_out/${R}_bench_f32.json | head -1
timeout -k 10 400 python bench.py --model adaattn --steps 40 > gpurun_out/${R}_bench_aa4.json 2> gpurun_out/${R}_bench_aa4.err || exit 8
python tools/show_bench.py gpurun_out/${R}_bench_aa4.json | head -1
timeout -k 10 600 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 20 --prof-steps 3 --cpu-steps 1 --cpu-warmup 0 --no-vgg19 > gpurun_out/${R}_bench_aa5.json 2> gpurun_out/${R}_bench_aa5.err || exit 9
python tools/show_bench.py gpurun_out/${R}_bench_aa5.json | head -1
VST_WGRAD_SIDE=0 VST_CONTENT_SIDE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof3 -o run -- \
  python3 bench.py --steps 10 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/${R}_prof3.log 2>&1 || exit 10
python tools/prof_summary.py gpurun_out/${R}_prof3 12 -shapes > gpurun_out/${R}_kernel_summary.txt 2>&1; cp gpurun_out/${R}_prof3/run_kernel_stats.csv gpurun_out/${R}_kernel_stats.csv
VST_WGRAD_SIDE=0 VST_CONTENT_SIDE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof5 -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 5 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/${R}_prof5.log 2>&1 || exit 11
python tools/prof_summary.py gpurun_out/${R}_prof5 7 -shapes > gpurun_out/${R}_adaattn_c5_kernel_summary.txt 2>&1; cp gpurun_out/${R}_prof5/run_kernel_stats.csv gpurun_out/${R}_adaattn_c5_kernel_stats.csv
rm -rf gpurun_out/${R}_prof3 gpurun_out/${R}_prof5
echo done
