#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export BENCH_MODES=3,35 BENCH_ONLY=res,aadec7
bash tools/pmc_wgrad.sh wgres || exit 3
export BENCH_MODES=4,36
bash tools/pmc_wgrad.sh wgres16 || exit 4
rm -rf gpurun_out/pmcb_*
