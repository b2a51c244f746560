#!/bin/bash
# build + profile the FETCH_SIZE/WRITE_SIZE calibration kernels (one gpurun step)
set -o pipefail
cd "$GRAFT_REPO_ROOT/tools/calib" || exit 1
hipcc --offload-arch=gfx950 -O2 -o hbm_calib hbm_calib.hip 2>/dev/null || exit 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/calib_$c -o run -- \
    tools/calib/hbm_calib > gpurun_out/calib_$c.log 2>&1 || exit 3
done
echo calib done
