#!/bin/bash
# residual-block data gradient: interior GEMM + border ring vs the padded grid (tests, config 3 / 4 A/B/A/B)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dgrad_ring.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05y_tests.log 2>&1 || { tail -30 gpurun_out/r05y_tests.log; exit 2; }
tail -1 gpurun_out/r05y_tests.log
for r in 1 0 1 0; do
  VST_PADOUT_RING=$r timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r05y_c3_$r.json 2>/dev/null || exit 5
  echo "ring=$r"; python tools/show_bench.py gpurun_out/r05y_c3_$r.json | head -1
done
for r in 1 0; do
  VST_PADOUT_RING=$r timeout -k 10 400 python bench.py --model adaattn --steps 40 --no-cpu-baseline --no-vgg19 > gpurun_out/r05y_aa4_$r.json 2>/dev/null || exit 6
  echo "ring=$r"; python tools/show_bench.py gpurun_out/r05y_aa4_$r.json | head -1
done
