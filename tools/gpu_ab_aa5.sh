cd $GRAFT_REPO_ROOT
L=video-style-transfer_amd/vst/libvst_hip.so
cp $L /tmp/libvst_main.so || exit 2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/hi_tests.log 2>&1 || exit 4
i=0
for lib in /tmp/libvst_main.so gpurun_tmp/libvst_head.so /tmp/libvst_main.so gpurun_tmp/libvst_head.so; do
  i=$((i+1)); cp $lib $L || exit 2
  timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 2 --no-cpu-baseline --no-vgg19 > gpurun_out/hi_aa5_$i.json 2>/dev/null || { cp /tmp/libvst_main.so $L; exit 5; }
done
cp /tmp/libvst_main.so $L
echo ok
