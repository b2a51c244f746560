#!/bin/bash
# golden margins of the channel-blocked order inside the stylizer, with and without A-direct tiles
cd $GRAFT_REPO_ROOT
export POLICY_DETAIL=1
VST_KBLOCK=2 timeout -k 10 200 python tools/policy_check.py bf16x6 > gpurun_out/kbp_ad.log 2>&1 || exit 3
VST_KBLOCK=2 VST_AD64=0 VST_AD128=0 VST_AD192=0 VST_AD256=0 timeout -k 10 200 python tools/policy_check.py bf16x6 > gpurun_out/kbp_noad.log 2>&1 || exit 3
VST_KBLOCK=2 timeout -k 10 200 python tools/policy_check.py f32 > gpurun_out/kbp_f32.log 2>&1 || exit 3
echo ok
