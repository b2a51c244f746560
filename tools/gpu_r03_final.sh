#!/bin/bash
# round-3 measurement of the tree on one box: the GPU suite, smoke(), PMC traffic + MFMA-busy passes
# of the headline step (installed under profiles/ so bench.py attaches them), the headline line (with
# CPU baseline, float64-gated full-size parity and the VGG19 sub-metric), the strict-f32 line, the
# config-4 AdaAttN line, and the rocprofv3 kernel summary of the headline command
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_fin_tests.log 2>&1 || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_fin_smoke.log 2>&1 || exit 3
bash tools/pmc_r02.sh reconet > gpurun_out/fin_pmc.log 2>&1 || exit 4
python tools/pmc_traffic.py reconet gpurun_out/r03_traffic_reconet.json --after-marker > gpurun_out/fin_traffic.log 2>&1 || exit 4
cp gpurun_out/r03_traffic_reconet.json profiles/ || exit 4
bash tools/pmc_busy_r02.sh reconet > gpurun_out/fin_busy.log 2>&1 || exit 4
python tools/pmc_busy.py reconet gpurun_out/r03_mfma_busy_reconet.json > gpurun_out/fin_busy2.log 2>&1 || exit 4
timeout -k 10 500 python bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || exit 5
timeout -k 10 300 python bench.py --gemm f32 --steps 60 --no-cpu-baseline > gpurun_out/r03_bench_f32.json 2> gpurun_out/r03_bench_f32.err || exit 6
timeout -k 10 400 python bench.py --model adaattn --steps 40 > gpurun_out/r03_bench_aa4.json 2> gpurun_out/r03_bench_aa4.err || exit 7
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin_prof -o run -- \
  python3 bench.py --steps 20 --prof-steps 5 --no-cpu-baseline --no-vgg19 > gpurun_out/fin_prof.log 2>&1 || exit 8
echo done
