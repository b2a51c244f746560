#!/bin/bash
# golden margins of the channel-blocked order inside the stylizer (everywhere / residual blocks only)
cd $GRAFT_REPO_ROOT
export POLICY_DETAIL=1
VST_KBLOCK=res timeout -k 10 200 python tools/policy_check.py bf16x6 f32 > gpurun_out/kbp_res.log 2>&1 || exit 3
echo ok
