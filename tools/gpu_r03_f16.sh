#!/bin/bash
# fp16 policy at mid size and at config 5 with full-size parity, the NaN locator first
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python tools/nan_diag.py > gpurun_out/r03_nan.log 2>&1 || exit 4
timeout -k 10 600 python -u -m pytest tests/test_gpu_adaattn.py -v -s --timeout 300 --timeout-method thread \
  -k "midsize" > gpurun_out/r03_f16b_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 3; fi
timeout -k 10 600 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --prof-steps 2 --cpu-steps 1 --cpu-warmup 0 --no-vgg19 --gemm f16 > gpurun_out/r03_c5_f16.json 2> gpurun_out/r03_c5_f16.err || exit 6
echo done
