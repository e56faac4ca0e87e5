#!/usr/bin/env python3
"""VGPR / SGPR / spill / LDS counts of the kernels in a HIP object's gfx950
code object (the AMDGPU metadata notes): python tools/kernel_regs.py [obj] [substr...]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
obj = sys.argv[1] if len(sys.argv) > 1 else "build/obj/render.o"
subs = sys.argv[2:] or ["wf_", "trace_kernel"]
with tempfile.TemporaryDirectory() as d:
    co, fb = os.path.join(d, "co"), os.path.join(d, "fatbin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(d, "x.o")],
                   check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--input={fb}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}", "--unbundle"], check=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
for blk in notes.split("- .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk)
    if not name or not any(s in name.group(1) for s in subs):
        continue
    g = {k: re.search(rf"\.{k}:\s+(\S+)", blk) for k in ("vgpr_count", "sgpr_count", "vgpr_spill_count",
                                                        "sgpr_spill_count", "group_segment_fixed_size",
                                                        "private_segment_fixed_size")}
    print(name.group(1)[:70], {k: (v.group(1) if v else None) for k, v in g.items()})
