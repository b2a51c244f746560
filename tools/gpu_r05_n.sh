#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/f16_sensitivity.py 64x128 128x256 > gpurun_out/r05n_sens.log 2>&1
rc=$?; tail -c 6000 gpurun_out/r05n_sens.log; exit $rc
