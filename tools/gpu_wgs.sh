#!/bin/bash
cd $GRAFT_REPO_ROOT
for m in 1 2 3 4 6; do
  echo "SMUL=$m"
  VST_WGRAD_SMUL=$m timeout -k 10 100 python tools/gemm_modes.py --modes bf16x3 --what wgrad 2>&1 | grep -v amdgpu || exit 2
done
