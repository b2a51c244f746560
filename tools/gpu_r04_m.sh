#!/bin/bash
# split-K diagnosis: split vs unsplit halo launches over the mid-size AdaAttN shapes, and the f16
# mid-size / reduced-policy tests with the weight-gradient side stream off
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/split_diag.py > gpurun_out/r04m_diag.log 2>&1 || { tail -20 gpurun_out/r04m_diag.log; exit 3; }
grep -c "<--" gpurun_out/r04m_diag.log; grep "<--\|worst" gpurun_out/r04m_diag.log | head -40
VST_WGRAD_SIDE=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_adaattn.py -k 'reduced_policy or midsize' -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04m_noside.log 2>&1
echo "noside rc=$?"; grep "policy: loss\|step: loss\|own-norm worst\|passed\|failed" gpurun_out/r04m_noside.log
echo done
