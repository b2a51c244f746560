#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/ddp_diag.py reconet 2>&1 | grep -v Gloo | grep -v amdgpu.ids | grep -v socket.cpp
echo "== side streams off"
VST_WGRAD_SIDE=0 VST_CONTENT_SIDE=0 timeout -k 10 200 python tools/ddp_diag.py reconet 2>&1 | grep -v Gloo | grep -v amdgpu.ids | grep -v socket.cpp
