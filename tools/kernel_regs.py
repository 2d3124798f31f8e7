#!/usr/bin/env python3
"""Per-kernel register counts of a built liboc_engine.so (the gfx950 code object's metadata):
  python tools/kernel_regs.py LIB.so [substring ...]
Prints name, VGPRs, SGPRs, LDS bytes for the kernels whose (mangled) names contain every
substring.  Uses the ROCm LLVM tools (llvm-objcopy, clang-offload-bundler, llvm-readelf)."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    lib, subs = sys.argv[1], sys.argv[2:]
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat"), os.path.join(d, "co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True, text=True).stdout
    for blk in notes.split("- .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk)
        if not name or not all(s in name.group(1) for s in subs):
            continue
        g = lambda k: (re.search(r"\.%s:\s+(\d+)" % k, blk) or [None, "?"])[1]
        print("%-90s vgpr %4s sgpr %4s lds %6s" % (name.group(1)[:90], g("vgpr_count"), g("sgpr_count"),
                                                  g("group_segment_fixed_size")))


if __name__ == "__main__":
    main()
