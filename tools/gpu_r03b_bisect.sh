#!/bin/bash
# conv parity cases under the run-time switches of the in-tree build
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T="tests/test_gpu_parity.py::test_conv_fwd_bwd"
for e in "VST_PF2=1" "VST_PF2=0"; do
  echo "== $e" >> gpurun_out/bisect.log
  env $e timeout -k 10 600 python -u -m pytest $T -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf 2>&1 | grep -E "passed|failed|FAILED" >> gpurun_out/bisect.log
done
echo done
