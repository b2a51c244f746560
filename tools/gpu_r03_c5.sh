#!/bin/bash
# config-5 precision decision: the config-5 step under bf16x3 (and fp32-class bf16x6) with full-size parity
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for G in bf16x3 bf16x6; do
timeout -k 10 900 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --prof-steps 2 --cpu-steps 1 --cpu-warmup 0 --no-vgg19 --gemm $G > gpurun_out/r03_c5_$G.json 2> gpurun_out/r03_c5_$G.err || exit 6
done
echo done
