#!/bin/bash
# config-5 precision decision: fp16 unit + mid-size tests, then the config-5 step under each
# candidate policy with full-size parity (one box, one call: comparable timings)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_adaattn.py -v -s --timeout 300 --timeout-method thread \
  -k "(conv_fwd_bwd and f16) or midsize" > gpurun_out/r03_f16_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 3; fi
for G in f16 bf16x3 bf16; do
timeout -k 10 600 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --prof-steps 2 --cpu-steps 1 --cpu-warmup 0 --no-vgg19 --gemm $G > gpurun_out/r03_c5_$G.json 2> gpurun_out/r03_c5_$G.err || exit 6
done
echo done
