#!/bin/bash
# per-tensor gradient norms of the aa_step golden step (bf16 policy): two-stage prefetch off, conv only,
# weight gradient only, both
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
VST_PF2=0 timeout -k 10 300 python tools/pf2_diag.py bf16 gpurun_out/pf2d_off.json > gpurun_out/pf2d.log 2>&1 || exit 3
VST_PF2=1 VST_WPF2=0 timeout -k 10 300 python tools/pf2_diag.py bf16 gpurun_out/pf2d_conv.json >> gpurun_out/pf2d.log 2>&1 || exit 3
VST_PF2=0 VST_WPF2=1 timeout -k 10 300 python tools/pf2_diag.py bf16 gpurun_out/pf2d_wgrad.json >> gpurun_out/pf2d.log 2>&1 || exit 3
echo done
