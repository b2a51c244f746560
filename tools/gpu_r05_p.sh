#!/bin/bash
# bf16x3 on the halo kernel (the f16 policy's loss-network forward), f16 order-insensitivity and 512x1024 tests
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -s > gpurun_out/r05p_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05p_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r05p_tests.log | head -30; exit 2; }
grep -E "^f16 (64|128|512)|f16 policy|f16 128x256|f16 256x512" gpurun_out/r05p_tests.log | head -30
for sk in 1 0 1 0; do
  VST_SPLITK=$sk timeout -k 10 400 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/r05p_aa5_$sk.json 2> gpurun_out/r05p_aa5.err || exit 9
  echo "SPLITK=$sk"; python tools/show_bench.py gpurun_out/r05p_aa5_$sk.json | head -3
done
timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r05p_c3.json 2>/dev/null || exit 5
python tools/show_bench.py gpurun_out/r05p_c3.json | head -3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05p_prof5 -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 3 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r05p_prof5.log 2>&1 || exit 6
python tools/prof_summary.py gpurun_out/r05p_prof5 5 > gpurun_out/r05p_c5_summary.txt 2>&1; head -40 gpurun_out/r05p_c5_summary.txt
