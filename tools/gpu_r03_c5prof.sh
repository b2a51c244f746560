#!/bin/bash
# config 5 (AdaAttN, B=8, 512x1024, f16 policy): its own PMC traffic / MFMA-busy summaries, the
# bench line with full-size parity, and the rocprofv3 kernel summary of the same command
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/pmc_r02.sh adaattn_c5 > gpurun_out/c5_pmc.log 2>&1 || exit 3
python tools/pmc_traffic.py adaattn_c5 gpurun_out/r03_traffic_adaattn_c5.json --after-marker > gpurun_out/c5_traffic.log 2>&1 || exit 3
cp gpurun_out/r03_traffic_adaattn_c5.json profiles/ || exit 3
bash tools/pmc_busy_r02.sh adaattn_c5 > gpurun_out/c5_busy.log 2>&1 || exit 4
python tools/pmc_busy.py adaattn_c5 gpurun_out/r03_mfma_busy_adaattn_c5.json > gpurun_out/c5_busy2.log 2>&1 || exit 4
timeout -k 10 600 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 20 --prof-steps 3 --cpu-steps 1 --cpu-warmup 0 --no-vgg19 > gpurun_out/r03_bench_aa5.json 2> gpurun_out/r03_bench_aa5.err || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5_prof -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 5 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/c5_prof.log 2>&1 || exit 6
echo done
