#!/bin/bash
# which VGG19 slices of the f16 policy's loss-network forward need bf16x3: accuracy and config-5 time
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V="f16 ship-lossnet1 ship-lossnet12 ship-lossnet123 ship-lossnet345 ship-lossnet1234"
timeout -k 10 700 python -u tools/f16_sensitivity.py 64x128 128x256 $V > gpurun_out/r05t_sens.log 2>&1 || { tail -20 gpurun_out/r05t_sens.log; exit 2; }
python - <<'PY'
import json
for line in open('gpurun_out/r05t_sens.log'):
    if not line.startswith('{'): continue
    for size, v in json.loads(line).items():
        for var, r in v.items():
            print(size, var, 'loss %.1e' % r['loss_rel'], 'cos_ref', ['%.6f' % c for c in r['whole_cos_vs_ref']], 'pair %.6f' % r['whole_cos_pair'], r['worst_own'][:2])
PY
for v in $V f16; do
  timeout -k 10 400 python tools/policy_bench.py $v --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/r05t_aa5_$v.json 2> gpurun_out/r05t_aa5.err || { tail -5 gpurun_out/r05t_aa5.err; exit 9; }
  echo "$v"; python tools/show_bench.py gpurun_out/r05t_aa5_$v.json | head -1
done
