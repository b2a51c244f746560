#!/bin/bash
# round-3 closing measurement of the final build: GPU suite + smoke(), headline line (driver
# defaults), config 4 and config 5 lines (full-size parity), rocprofv3 summary of the config-5 step
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/final_tests.log 2>&1 || { tail -40 gpurun_out/final_tests.log; exit 4; }
tail -2 gpurun_out/final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 5
timeout -k 10 600 python bench.py > gpurun_out/r03c_bench.json 2> gpurun_out/r03c_bench.err || exit 6
python tools/show_bench.py gpurun_out/r03c_bench.json | head -3
timeout -k 10 400 python bench.py --model adaattn --steps 40 > gpurun_out/r03c_bench_aa4.json 2> gpurun_out/r03c_bench_aa4.err || exit 7
timeout -k 10 600 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 20 --prof-steps 3 --cpu-steps 1 --cpu-warmup 0 --no-vgg19 > gpurun_out/r03c_bench_aa5.json 2> gpurun_out/r03c_bench_aa5.err || exit 8
python tools/show_bench.py gpurun_out/r03c_bench_aa5.json | head -3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03c_prof5 -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 5 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/r03c_prof5.log 2>&1 || exit 10
python tools/prof_summary.py gpurun_out/r03c_prof5 12 > gpurun_out/r03c_adaattn_c5_kernel_summary.txt 2>&1
echo done
