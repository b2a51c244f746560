#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad_halo.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05m_wh.log 2>&1 || { tail -40 gpurun_out/r05m_wh.log; exit 3; }
tail -1 gpurun_out/r05m_wh.log
for i in 1 2; do
  (cd variants/r4 && timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > ../../gpurun_out/r05m_r4_$i.json 2>/dev/null) || exit 5
  python tools/show_bench.py gpurun_out/r05m_r4_$i.json | head -1
  timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r05m_head_$i.json 2> gpurun_out/r05m_head.err || exit 6
  python tools/show_bench.py gpurun_out/r05m_head_$i.json | head -1
done
VST_WGRAD_SIDE=0 VST_CONTENT_SIDE=0 timeout -k 10 300 python tools/conv_breakdown.py reconet 3 > gpurun_out/r05m_breakdown.txt 2>&1 || exit 7
cat gpurun_out/r05m_breakdown.txt
