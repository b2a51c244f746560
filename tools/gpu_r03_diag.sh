#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python tools/grad_diag.py --terms OTL,CL --nosink > gpurun_out/r03_gdiag_nosink.log 2>&1 || exit 3
timeout -k 10 200 python tools/grad_diag.py --terms OTL,CL --tag b1r > gpurun_out/r03_gdiag_b1r.log 2>&1 || exit 3
echo done
