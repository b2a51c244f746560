#!/bin/bash
# per-shape GEMM breakdown of the headline step (bf16x6) and the rocprofv3 kernel summary
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
VST_GEMM_POLICY=bf16x6 timeout -k 10 300 python tools/conv_breakdown.py reconet 3 > gpurun_out/r03_cb.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3_prof -o run -- \
  python3 bench.py --steps 20 --prof-steps 5 --no-cpu-baseline --no-vgg19 > gpurun_out/c3_prof.log 2>&1 || exit 4
echo done
