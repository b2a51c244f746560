#!/bin/bash
# f16 mid-size step vs the oracle, per-tensor errors, split (default) vs libnosplit
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in default nosplit; do
  if [ $v = default ]; then LP=""; else LP=video-style-transfer_amd/vst/variants/lib$v.so; fi
  VST_LIB_PATH=$LP timeout -k 10 300 python -u -c "
import sys, json; sys.argv=['x']; sys.path[:0]=['tools']
import f16_parity_diag as d, torch
torch.set_num_threads(16)
r = d.step_vs_oracle('f16', 1, 128, 256, k=14)
print('$v', json.dumps(r))
" > gpurun_out/r04n_$v.log 2>&1 || { tail -20 gpurun_out/r04n_$v.log; exit 3; }
  tail -1 gpurun_out/r04n_$v.log
done
