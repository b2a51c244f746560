#!/bin/bash
# measured halo block shapes: halo tests, headline + config-5 step timings, rocprofv3 kernel summaries
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_halo.py tests/test_gpu_scaler.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04e_halo.log 2>&1 || { tail -40 gpurun_out/r04e_halo.log; exit 3; }
tail -2 gpurun_out/r04e_halo.log
timeout -k 10 300 python bench.py --steps 100 --prof-steps 1 --no-cpu-baseline --no-vgg19 > gpurun_out/r04e_c3.json 2>/dev/null || exit 7
python tools/show_bench.py gpurun_out/r04e_c3.json | head -1
timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 3 --prof-steps 1 --no-cpu-baseline --no-vgg19 > gpurun_out/r04e_c5.json 2>/dev/null || exit 6
python tools/show_bench.py gpurun_out/r04e_c5.json | head -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04e_prof3 -o run -- \
  python3 bench.py --steps 10 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r04e_prof3.log 2>&1 || exit 10
python tools/prof_summary.py gpurun_out/r04e_prof3 12 -shapes > gpurun_out/r04e_c3_kernel_summary.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04e_prof5 -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 5 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r04e_prof5.log 2>&1 || exit 11
python tools/prof_summary.py gpurun_out/r04e_prof5 7 -shapes > gpurun_out/r04e_c5_kernel_summary.txt 2>&1
rm -rf gpurun_out/r04e_prof3 gpurun_out/r04e_prof5
echo done
