#!/bin/bash
# VGPR / spill / scratch per kernel of one HIP source, with extra compile flags:
#   tools/ru.sh kernels_persist.hip -DWRNN_PERSIST_PART=1 -mllvm -amdgpu-sched-strategy=iterative-ilp
f=$1; shift
cd "$(dirname "$0")/../real-time-voice-cloning_amd/csrc"
/opt/rocm/bin/hipcc -std=c++17 -O3 -fno-slp-vectorize --offload-arch=gfx950 -I../../include -c "$f" -o /tmp/ru_$$.o "$@" \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import sys, re
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m: cur = [m.group(1), {}]; rows.append(cur); continue
    for key in ("VGPRs:", "AGPRs:", "VGPRs Spill:", "ScratchSize [bytes/lane]:", "Occupancy [waves/SIMD]:"):
        if key in line and cur is not None:
            cur[1][key.rstrip(":")] = line.split(key)[1].split()[0]
for n, d in rows:
    if "k_persist" in n or "wide" in n:
        print(n[:60], " ".join(f"{k}={v}" for k, v in d.items()))'
rm -f /tmp/ru_$$.o
