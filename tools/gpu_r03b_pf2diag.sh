#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for pf in 1 0; do
  VST_PF2=$pf timeout -k 10 300 python tools/pf2_diag.py bf16 gpurun_out/pf2diag_bf16_$pf.json > gpurun_out/pf2diag_$pf.log 2>&1 || exit 3
  VST_PF2=$pf VST_WKD2=1 VST_KD2=1 timeout -k 10 300 python -c "print('ok')" > /dev/null || exit 3
done
echo done
