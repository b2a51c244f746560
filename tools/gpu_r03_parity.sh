#!/bin/bash
# round-3 parity evidence: stylizer block chain per term, mid-size AdaAttN tests, then the
# config-3 headline line (fp64-gated full-size parity), config-4 and config-5 lines with the
# AdaAttN full_size_parity blocks
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_adaattn.py -v -s --timeout 300 --timeout-method thread \
  -k "block_chain or midsize" > gpurun_out/r03_par_tests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 3; fi
timeout -k 10 400 python bench.py --no-vgg19 --steps 60 > gpurun_out/r03_par_c3.json 2> gpurun_out/r03_par_c3.err || exit 4
timeout -k 10 400 python bench.py --model adaattn --steps 20 --prof-steps 3 --no-vgg19 > gpurun_out/r03_par_c4.json 2> gpurun_out/r03_par_c4.err || exit 5
timeout -k 10 900 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --prof-steps 2 --cpu-steps 1 --no-vgg19 > gpurun_out/r03_par_c5.json 2> gpurun_out/r03_par_c5.err || exit 6
echo done
