#!/bin/bash
# GPU tests + per-layer GEMM timing + parity bench (usage: tools/gpu_quick.sh [gemm_modes args])
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/gemm_modes.py --modes ${MODES:-bf16x3,bf16x6} "$@" > gpurun_out/modes.log 2>&1 || { echo "gemm_modes failed"; tail -5 gpurun_out/modes.log; exit 2; }
bash tools/gpu_run.sh ${POLS:-parity}
