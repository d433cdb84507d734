#!/bin/bash
# Per-kernel resource usage (VGPRs, SGPRs, scratch, occupancy) of one HIP source,
# from the compiler's kernel-resource-usage remarks.  Usage: tools/regs.sh k_rtcsm.hip
cd "$(dirname "$0")/../my-lidar-graph-slam_amd/csrc" || exit 2
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -fno-fast-math -fno-gpu-rdc \
    -I../../include -I. -c -o /tmp/regs_probe.o "$1" -Rpass-analysis=kernel-resource-usage 2>&1 |
  python3 -c '
import re, sys
cur = None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        n = m.group(1); k = re.search(r"(k_\w+?)(?:ILi(\d+)E)?E", n)
        cur = (k.group(1) + (f"<{k.group(2)}>" if k.group(2) else "")) if k else n[:40]
        print(); print(f"{cur:22s}", end="")
        continue
    for key in ("VGPRs", "TotalSGPRs", "ScratchSize \[bytes/lane\]", "Occupancy \[waves/SIMD\]", "LDS Size \[bytes/block\]"):
        m = re.search(key + r": (\d+)", line)
        if m: print(f" {key.split()[0]}={m.group(1)}", end="")
print()'
