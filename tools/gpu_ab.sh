#!/bin/bash
# A/B of library builds of THIS tree (csrc/Makefile VARIANT_FLAGS, same sources -> same build id) on one
# box, interleaved:  tools/gpu_ab.sh TAG "BENCH ARGS" LIB1 LIB2 ...   (each LIB a path under vst/; the
# in-tree library is "main").  Lines go to gpurun_out/ab_TAG_<i>_<lib>.json.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; ARGS=$2; shift 2
for rep in 1 2; do
  for lib in "$@"; do
    p=video-style-transfer_amd/vst/$lib
    [ "$lib" = main ] && p=video-style-transfer_amd/vst/libvst_hip.so
    out=gpurun_out/ab_${TAG}_${rep}_${lib%.so}.json
    VST_LIB_PATH=$p timeout -k 10 300 python bench.py $ARGS > $out 2> ${out%.json}.err
    rc=$?; case $rc in 0) ;; *) echo "bench rc=$rc ($lib)"; exit 9;; esac
    python -c "import json,sys; d=json.loads(open('$out').read().strip().splitlines()[-1]); print('$rep $lib', round(d['value'],2), round(d['ms_per_step'],2))"
  done
done
