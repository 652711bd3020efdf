#!/usr/bin/env python3
"""VGPR / spill / scratch per kernel of the product source (device-only compile).
  python tools/kres.py [filter] [-- extra hipcc flags]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
argv = sys.argv[1:]
extra = argv[argv.index("--") + 1:] if "--" in argv else []
filt = argv[0] if argv and argv[0] != "--" else ""
with tempfile.TemporaryDirectory() as d:
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++20", "--offload-arch=gfx950", f"-I{ROOT}/include",
                    "--cuda-device-only", "-S", "-o", f"{d}/k.s", f"{ROOT}/a3-reliable-transport_amd/csrc/crc32_kernels.hip",
                    *extra], check=True)
    s = open(f"{d}/k.s").read()
meta = s[s.find("amdhsa.kernels"):]
for b in meta.split("  - .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", b).group(1)
    if filt not in name:
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", b) or [None, None])[1]  # noqa: E731
    print(f"{name[:80]:80s} vgpr {g('vgpr_count')} spill {g('vgpr_spill_count')} scratch {g('private_segment_fixed_size')}")
