"""bench.py under a policy variant of tools/f16_sensitivity.py (registered before bench parses
--gemm):  python tools/policy_bench.py <variant> <bench.py arguments...>   (GPU)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-style-transfer_amd"), os.path.join(REPO, "tools")]

import f16_sensitivity  # noqa: E402

if __name__ == "__main__":
    name = f16_sensitivity.register(sys.argv[1])
    import bench

    sys.argv = ["bench.py", *sys.argv[2:], "--gemm", name]
    bench.main()
