#!/usr/bin/env python3
"""VGPR / spill / LDS usage of kernels in a hipcc -save-temps .s file (AMDGPU metadata).
usage: kernel_regs.py file.s [substring]"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
meta = s[s.index("amdhsa.kernels:"):]
for ent in re.split(r"\n  - ", meta)[1:]:
    name = re.search(r"\.name:\s+(\S+)", ent)
    if not name or pat not in name.group(1):
        continue
    f = {k: re.search(rf"\.{k}:\s+(\d+)", ent) for k in
         ("vgpr_count", "vgpr_spill_count", "sgpr_count", "group_segment_fixed_size")}
    print(name.group(1), *(f"{k}={v.group(1)}" for k, v in f.items() if v))
