"""Per-kernel VGPR / spill / SGPR / LDS figures from a built object's gfx950 code object.

    python tools/kernel_resources.py [object.o] [name-substring ...]

Reads the .hip_fatbin section of an object built by ac-solver-caltech_amd/build.py (no GPU,
no rebuild), unbundles the gfx950 code object and prints its kernel metadata notes.
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    obj = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "..", "ac-solver-caltech_amd", "build",
                                                            "acx_kernels.hip.o")
    pats = sys.argv[2:]
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "k.co")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(d, "x")])
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
        notes = subprocess.check_output([f"{LLVM}/llvm-readelf", "--notes", co], text=True)
    for blk in notes.split("- .agpr_count")[1:]:
        g = lambda k: (re.search(rf"\.{k}:\s+(\S+)", blk) or [None, "?"])[1]
        name = g("name")
        if pats and not any(p in name for p in pats):
            continue
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        print(f"vgpr {g('vgpr_count'):>4} spill {g('vgpr_spill_count'):>3} sgpr {g('sgpr_count'):>3} "
              f"lds {g('group_segment_fixed_size'):>6}  {dem[:110]}")


if __name__ == "__main__":
    main()
