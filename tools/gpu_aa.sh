#!/bin/bash
# AdaAttN benches: config-4 shape (B=4, 256x512) under the parity policy; config-5 shape (B=8, 512x1024, bf16)
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --model adaattn --steps 5 --warmup 2 --no-cpu-baseline --no-vgg19 --gemm ${GEMM4:-parity} > gpurun_out/aa_c4.log 2>&1 || { echo "c4 failed"; tail -5 gpurun_out/aa_c4.log; exit 2; }
tail -1 gpurun_out/aa_c4.log
timeout -k 10 400 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 2 --warmup 1 --no-cpu-baseline --no-vgg19 --gemm bf16 > gpurun_out/aa_c5.log 2>&1 || { echo "c5 failed"; tail -5 gpurun_out/aa_c5.log; exit 3; }
tail -1 gpurun_out/aa_c5.log
