cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_halo.py tests/test_gpu_wgrad_halo.py tests/test_gpu_streams.py -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf --tb=short > gpurun_out/r06c_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06c_tests.log
case $rc in 0|1) ;; *) exit 9;; esac
timeout -k 10 600 python -u -m pytest tests/test_gpu_adaattn.py -q -k "f16 or 512" --timeout 300 --timeout-method thread -p no:cacheprovider -rf --tb=short -s > gpurun_out/r06c_f16tests.log 2>&1; rc=$?; echo "f16 tests rc=$rc"; grep -E "512x1024|passed|failed" gpurun_out/r06c_f16tests.log | tail -8
case $rc in 0|1) ;; *) exit 9;; esac
bash tools/gpu_ab.sh c5 "--model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19" main libvst_hip_ad1.so libvst_hip_ad8.so
