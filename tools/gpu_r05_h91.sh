#!/bin/bash
# 9 x 1 halo (the kw-unfolded 9x9 layers): full GPU suite, config 3 A/B/A/B on the forward's K order
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo.py -x -q -k halo91 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05h91_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05h91_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r05h91_tests.log | head -30; exit 2; }
for r in 1 0 1 0; do
  VST_HALO91=$r timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r05h91_c3_$r.json 2>/dev/null || exit 5
  echo "halo91=$r"; python tools/show_bench.py gpurun_out/r05h91_c3_$r.json | head -2
done
