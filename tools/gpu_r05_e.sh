#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad_halo.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05e_wh.log 2>&1 || { tail -40 gpurun_out/r05e_wh.log; exit 3; }
tail -1 gpurun_out/r05e_wh.log
BENCH_MODES=3,35,4,36 BENCH_ONLY=res,aadec timeout -k 10 300 python tools/wgrad_bench.py > gpurun_out/r05e_wbench.txt 2>&1 || { cat gpurun_out/r05e_wbench.txt; exit 7; }
cat gpurun_out/r05e_wbench.txt
export BENCH_MODES=3,35 BENCH_ONLY=res
bash tools/pmc_wgrad.sh wgres || exit 4
rm -rf gpurun_out/pmcb_*
