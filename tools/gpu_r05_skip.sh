#!/bin/bash
# residual skip gradient accumulated in conv1's data gradient: new tests, the ReCoNet parity / golden
# tests, then config 3 A/B/A/B with VST_SKIP_ACCUM on / off (one box)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_skipgrad.py tests/test_gpu_parity.py tests/test_gpu_streams.py tests/test_gpu_abi.py tests/test_gpu_ddp.py > gpurun_out/skip_tests.log 2>&1 || { tail -40 gpurun_out/skip_tests.log; exit 4; }
tail -2 gpurun_out/skip_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/skip_on_$i.json 2>/dev/null || exit 5
  python tools/show_bench.py gpurun_out/skip_on_$i.json 2>/dev/null | head -1
  VST_SKIP_ACCUM=0 timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/skip_off_$i.json 2>/dev/null || exit 6
  python tools/show_bench.py gpurun_out/skip_off_$i.json 2>/dev/null | head -1
done
echo done
