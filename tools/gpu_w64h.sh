cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wgrad_halo.py tests/test_gpu_elementwise.py tests/test_gpu_abi.py tests/test_gpu_streams.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/w64h_tests.log 2>&1 || { tail -30 gpurun_out/w64h_tests.log; exit 4; }
tail -2 gpurun_out/w64h_tests.log
VST_WGRAD_SIDE=0 VST_CONTENT_SIDE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/w64h_prof3 -o run -- \
  python3 bench.py --steps 10 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/w64h_prof3.log 2>&1 || exit 10
python tools/prof_summary.py gpurun_out/w64h_prof3 12 -shapes > gpurun_out/w64h_kernel_summary.txt 2>&1
grep wgrad2 gpurun_out/w64h_kernel_summary.txt
rm -rf gpurun_out/w64h_prof3
timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/w64h_bench.json 2>/dev/null || exit 6
python tools/show_bench.py gpurun_out/w64h_bench.json | head -1
