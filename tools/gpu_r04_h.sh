#!/bin/bash
# tuned halo occupancy: new GPU tests (DP through HIP, AdaAttN API, halo, AdaAttN incl. the decoder's
# K order), config-5 parity measurements, headline / config-5 timings and the config-5 kernel summary
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_adaattn_api.py tests/test_gpu_halo.py tests/test_gpu_adaattn.py tests/test_gpu_scaler.py -q -rA --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04h_tests.log 2>&1
rc=$?
grep -E "passed|failed|buckets|PASSED.*ddp|FAILED" gpurun_out/r04h_tests.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 4
timeout -k 10 300 python bench.py --steps 100 --prof-steps 1 --no-cpu-baseline --no-vgg19 > gpurun_out/r04h_c3.json 2>/dev/null || exit 7
python tools/show_bench.py gpurun_out/r04h_c3.json | head -1
timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 3 --prof-steps 1 --no-cpu-baseline --no-vgg19 > gpurun_out/r04h_c5.json 2>/dev/null || exit 6
python tools/show_bench.py gpurun_out/r04h_c5.json | head -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04h_prof5 -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 5 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r04h_prof5.log 2>&1 || exit 11
python tools/prof_summary.py gpurun_out/r04h_prof5 7 -shapes > gpurun_out/r04h_c5_kernel_summary.txt 2>&1
rm -rf gpurun_out/r04h_prof5
timeout -k 10 600 python -u tools/f16_parity_diag.py f16 bf16 > gpurun_out/r04h_f16diag.json 2> gpurun_out/r04h_f16diag.err || { tail -20 gpurun_out/r04h_f16diag.err; exit 5; }
echo done
