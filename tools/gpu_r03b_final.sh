#!/bin/bash
# round-3 closing measurement on one box: GPU suite, smoke(), headline PMC traffic + MFMA-busy passes
# (installed under profiles/ so bench.py attaches them), the headline line (CPU baseline, float64-gated
# full-size parity, VGG19 sub-metric), strict f32, config 4 and config 5 lines (with full-size parity),
# and rocprofv3 kernel summaries of the headline and config-5 commands
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03b_tests.log 2>&1 || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03b_smoke.log 2>&1 || exit 3
bash tools/pmc_r02.sh reconet > gpurun_out/r03b_pmc.log 2>&1 || exit 4
python tools/pmc_traffic.py reconet gpurun_out/r03_traffic_reconet.json --after-marker > gpurun_out/r03b_traffic.log 2>&1 || exit 4
cp gpurun_out/r03_traffic_reconet.json profiles/ || exit 4
bash tools/pmc_busy_r02.sh reconet > gpurun_out/r03b_busy.log 2>&1 || exit 4
python tools/pmc_busy.py reconet gpurun_out/r03_mfma_busy_reconet.json > gpurun_out/r03b_busy2.log 2>&1 || exit 4
timeout -k 10 500 python bench.py > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.err || exit 5
timeout -k 10 300 python bench.py --gemm f32 --steps 60 --no-cpu-baseline > gpurun_out/r03b_bench_f32.json 2> gpurun_out/r03b_bench_f32.err || exit 6
echo done
