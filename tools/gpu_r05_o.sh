#!/bin/bash
# 2x2 halo (phase-stacked layers), f16 split-K re-admitted, f16 policy's loss-network forward on bf16x3
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05o_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05o_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r05o_tests.log | head -30; exit 2; }
grep -E "f16.*(margin|cosine)" gpurun_out/r05o_tests.log | head
for kb in 1 0 1 0; do
  VST_KBLOCK_UP2=$kb timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r05o_c3_$kb.json 2>/dev/null || exit 5
  echo "KBLOCK_UP2=$kb"; python tools/show_bench.py gpurun_out/r05o_c3_$kb.json | head -3
done
for sk in 1 0; do
  VST_SPLITK=$sk timeout -k 10 400 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/r05o_aa5_$sk.json 2> gpurun_out/r05o_aa5.err || exit 9
  echo "SPLITK=$sk"; python tools/show_bench.py gpurun_out/r05o_aa5_$sk.json | head -3
done
timeout -k 10 600 python -u tools/f16_sensitivity.py 64x128 128x256 f16 > gpurun_out/r05o_sens.log 2>&1 || exit 10
python - <<'PY'
import json
for line in open('gpurun_out/r05o_sens.log'):
    if not line.startswith('{'): continue
    for size, v in json.loads(line).items():
        for var, r in v.items():
            print(size, var, 'loss %.1e' % r['loss_rel'], 'cos_ref', ['%.6f' % c for c in r['whole_cos_vs_ref']], 'pair %.6f' % r['whole_cos_pair'], r['worst_own'][:2])
PY
timeout -k 10 300 python -u tools/graph_ab.py 40 > gpurun_out/r05o_graph.log 2>&1; tail -5 gpurun_out/r05o_graph.log
