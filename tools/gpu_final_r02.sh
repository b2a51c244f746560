#!/bin/bash
# round-2 closing measurement on one box: PMC traffic + MFMA-busy passes of the timed-region launch
# mix (converted on the box and installed under profiles/ so bench.py attaches them), the headline
# bench line, the f32-policy line, and the rocprofv3 kernel summary of the headline command
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/pmc_r02.sh reconet > gpurun_out/fin_pmc.log 2>&1 || exit 3
python tools/pmc_traffic.py reconet gpurun_out/r02_traffic_reconet.json --after-marker > gpurun_out/fin_traffic.log 2>&1 || exit 3
cp gpurun_out/r02_traffic_reconet.json profiles/r02_traffic_reconet.json || exit 3
bash tools/pmc_busy_r02.sh reconet > gpurun_out/fin_busy.log 2>&1 || exit 4
python tools/pmc_busy.py reconet gpurun_out/r02_mfma_busy_reconet.json > gpurun_out/fin_busy2.log 2>&1 || exit 4
timeout -k 10 400 python bench.py > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err || exit 5
timeout -k 10 300 python bench.py --gemm f32 --steps 60 --no-cpu-baseline > gpurun_out/r02_bench_f32.json 2> gpurun_out/r02_bench_f32.err || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin_prof -o run -- \
  python3 bench.py --steps 20 --prof-steps 5 --no-cpu-baseline --no-vgg19 > gpurun_out/fin_prof.log 2>&1 || exit 7
echo done
