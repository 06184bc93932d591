#!/bin/bash
# Per-kernel register / LDS / scratch usage of the gfx950 code objects (compiler resource remarks),
# so a scratch spill is tracked alongside the profiles:  scripts/kernel_resources.sh > profiles/rNN_kernel_resources.txt
cd "$(dirname "$0")/../mopo_amd/csrc"
T=$(mktemp -d)
for f in *.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only $( [ "$f" = bnn.hip -o "$f" = actor.hip ] && echo -mllvm -pragma-unroll-threshold=262144) -Rpass-analysis=kernel-resource-usage \
    -c "$f" -o /dev/null > "$T/$f.txt" 2>&1 &
done
wait
cat "$T"/*.txt | python3 -c '
import re, sys
rows, fn = [], None
for line in sys.stdin:
    m = re.search(r"remark: (.*?)( \[-Rpass.*)?$", line.rstrip())
    if not m: continue
    r = m.group(1).strip()
    k = re.match(r"Function Name: (\S+)", r)
    if k:
        fn = k.group(1); rows.append([fn]); continue
    v = re.match(r"(VGPRs|AGPRs|ScratchSize|Occupancy|LDS Size|VGPRs Spill)( \[[^]]*\])?: (\S+)", r)
    if fn and v:
        rows[-1].append("%s=%s" % (v.group(1).replace(" ", "_"), v.group(3)))
for r in rows:
    print(r[0] + "\t" + "  ".join(r[1:]))
' | c++filt | sort
rm -rf "$T"
