"""Per-kernel VGPR / AGPR / SGPR / LDS / scratch from a device .s (amdhsa metadata):
python tools/kernel_regs.py file.s [name-substring]"""
import re
import sys

text = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for block in re.split(r"\n  - \.", text.split("amdhsa.kernels:")[-1]):
    name = re.search(r"\.name:\s+(\S+)", block)
    if not name or pat not in name.group(1):
        continue
    get = lambda k: (re.search(rf"\.{k}:\s+(\d+)", block) or [None, "?"])[1]  # noqa: E731
    print(f"vgpr {get('vgpr_count'):>4} agpr {get('agpr_count'):>4} sgpr {get('sgpr_count'):>4} "
          f"lds {get('group_segment_fixed_size'):>6} scratch {get('private_segment_fixed_size'):>4}  {name.group(1)[:110]}")
