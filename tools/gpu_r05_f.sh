#!/bin/bash
# halo wgrad in the step: GPU suite, wgrad bench incl. the row-split decoder shapes, config 3 and config 5
# lines with the 64-output decoder convs on the row-split GEMM (default) and on the halo kernel (VST_RSW=0)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
BENCH_MODES=3,35,4,36 BENCH_ONLY=aadec6,aadec7 timeout -k 10 300 python tools/wgrad_bench.py > gpurun_out/r05f_wbench.txt 2>&1 || { cat gpurun_out/r05f_wbench.txt; exit 7; }
cat gpurun_out/r05f_wbench.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05f_tests.log 2>&1 || { tail -60 gpurun_out/r05f_tests.log; exit 4; }
tail -2 gpurun_out/r05f_tests.log
timeout -k 10 400 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r05f_c3.json 2> gpurun_out/r05f_c3.err || exit 6
python tools/show_bench.py gpurun_out/r05f_c3.json | head -3
for rs in 1 0 1 0; do
VST_RSW=$rs timeout -k 10 400 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/r05f_aa5_$rs.json 2> gpurun_out/r05f_aa5.err || exit 9
echo "RSW=$rs"; python tools/show_bench.py gpurun_out/r05f_aa5_$rs.json | head -3
done
echo done
