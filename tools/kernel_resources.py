"""VGPR / spill / scratch metadata of the gfx950 kernels in a built object (video-style-transfer_amd/csrc/build/*.o).

    python tools/kernel_resources.py video-style-transfer_amd/csrc/build/wgrad_gemm.o [name-filter]
"""
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin/"
obj = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
with tempfile.TemporaryDirectory() as d:
    subprocess.check_call([LLVM + "llvm-objcopy", f"--dump-section=.hip_fatbin={d}/fb", obj])
    subprocess.check_call([LLVM + "clang-offload-bundler", "-type=o", "-targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                           f"-input={d}/fb", f"-output={d}/co", "-unbundle"])
    notes = subprocess.check_output([LLVM + "llvm-readelf", "--notes", f"{d}/co"], text=True)
for blk in notes.split("- .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if filt not in name:
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]  # noqa: E731
    dem = subprocess.check_output(["c++filt", name], text=True).strip().replace("(anonymous namespace)::", "")
    print(f"vgpr {g('vgpr_count'):>4} agpr {blk.split(chr(10))[0].split(':')[-1].strip():>4} spill {g('vgpr_spill_count'):>3} scratch {g('private_segment_fixed_size'):>4} "
          f"lds {g('group_segment_fixed_size'):>6}  {dem[:100]}")
