#!/bin/bash
# Print VGPR / spill / LDS / occupancy per kernel of a HIP source (compile-time remarks).
f=${1:-kernels_step.hip}
cd "$(dirname "$0")/../real-time-voice-cloning_amd/csrc"
/opt/rocm/bin/hipcc -std=c++17 -O3 -fno-slp-vectorize --offload-arch=gfx950 -I../../include -c "$f" -o /tmp/ru.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import sys, re
cur = None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m: cur = m.group(1); print(); print(cur[:70], end=" "); continue
    for key in ("VGPRs:", "VGPRs Spill:", "LDS Size [bytes/block]:", "Occupancy [waves/SIMD]:", "TotalSGPRs:"):
        if key in line:
            v = line.split(key)[1].split()[0]
            print(key.split()[0].replace(":", "") + ("Spill" if "Spill" in key else "") + "=" + v, end=" ")
print()'
