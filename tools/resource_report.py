"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks per kernel."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "rrin_amd/csrc/conv_mfma.hip"
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-Iinclude",
       "-Rpass-analysis=kernel-resource-usage", "--cuda-device-only", "-c", src, "-o", "/dev/null"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark: ([A-Za-z /\[\]]+?): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    name = re.sub(r"_ZN4rrin\d+", "", k)
    print(f"{name[:60]:60s} vgpr {v.get('VGPRs','?'):>4} agpr {v.get('AGPRs','?'):>4} "
          f"occ {v.get('Occupancy [waves/SIMD]','?')} sgpr_spill {v.get('SGPRs Spill','?')} "
          f"vgpr_spill {v.get('VGPRs Spill','?')} lds {v.get('LDS Size [bytes/block]','?')}")
