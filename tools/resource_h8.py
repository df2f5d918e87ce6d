"""Register / occupancy table of the conv3x3_h8_kernel instantiations from a
`-Rpass-analysis=kernel-resource-usage` log (usage: resource_h8.py LOG [P])."""
import re
import sys

rows, cur = {}, None
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|Occupancy \[waves/SIMD\]|VGPRs Spill|ScratchSize \[bytes/lane\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0] + ("S" if "Spill" in m.group(1) else "")] = int(m.group(2))
planes = sys.argv[2] if len(sys.argv) > 2 else "2"
for f, r in rows.items():
    m = re.search(r"conv3x3_h8_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELb(\d)ELi(\d+)E", f)
    if m and m.group(4) == planes:
        nw, wm, wn, p, epi, dma, sc = m.groups()
        print(f"NW{nw} WM{wm} WN{wn} P{p} EPI{epi} DMA{dma} sched{sc}: vgpr {r.get('VGPRs')} agpr {r.get('AGPRs')} "
              f"occ {r.get('Occupancy')} spill {r.get('VGPRsS')} scratch {r.get('ScratchSize')}")
