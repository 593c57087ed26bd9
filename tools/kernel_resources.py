"""Print VGPR / SGPR / LDS / occupancy / spills per kernel of libhicgat (hipcc remarks)."""
import re
import subprocess
import sys
import os

root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "hic-gnn_amd")
srcs = sys.argv[1:] or sorted(f for f in os.listdir(os.path.join(root, "csrc")) if f.endswith(".hip"))
for f in srcs:
    out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                          "-c", "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage", os.path.join(root, "csrc", f)],
                         capture_output=True, text=True).stderr
    cur = None
    info = {}
    for line in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = t.split(":", 1)[1].strip()
            info[cur] = {}
        elif cur and ":" in t:
            k, v = t.split(":", 1)
            info[cur][k.strip()] = v.strip()
    for k, v in info.items():
        name = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip().split("(")[0]
        print(f"{name[:60]:60s} vgpr {v.get('VGPRs','?'):>4} agpr {v.get('AGPRs','?'):>3} "
              f"occ {v.get('Occupancy [waves/SIMD]','?'):>2} lds {v.get('LDS Size [bytes/block]','?'):>6} "
              f"spill {v.get('VGPRs Spill','?')}/{v.get('SGPRs Spill','?')}")
