# Per-family durations, inter-kernel gaps and one step's launch list from a rocprofv3
# --kernel-trace CSV of a one-stream bench run (steps delimited by pack_g16_r32_kernel).
# usage: python3 tools/trace_steps.py <run_kernel_trace.csv>
import csv, collections, sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
def nm(r): return r['Kernel_Name'].split('(')[0].replace('void ','').replace('rrin::','')
idx=[i for i,r in enumerate(rows) if nm(r).startswith('pack_g16')]
S=10; s0=idx[-S]; seg=rows[s0:]
fam=collections.defaultdict(lambda:[0,0.0,0.0]); prev=None; gaps=0
for r in seg:
    st=int(r['Start_Timestamp']); en=int(r['End_Timestamp']); n=nm(r)
    fam[n][0]+=1; fam[n][1]+=(en-st)/1e3
    if prev is not None: g=max(st-prev,0); gaps+=g; fam[n][2]+=g/1e3
    prev=en
span=(int(seg[-1]['End_Timestamp'])-int(seg[0]['Start_Timestamp']))/1e3
print('span us/step %.1f  gaps us/step %.1f'%(span/S, gaps/1e3/S))
for n,(c,t,g) in sorted(fam.items(), key=lambda x:-x[1][1]): print(f'{n:45s} {c/S:5.1f} {t/S:8.1f} us  avg {t/c:6.1f}  gap-before {g/S:6.1f}')
# per-launch list of one step
print('--- one step (dur us, gap us, grid, wg)')
one=rows[idx[-2]:idx[-1]]; prev=None
for r in one:
    st=int(r['Start_Timestamp']); en=int(r['End_Timestamp'])
    g=(st-prev)/1e3 if prev else 0; prev=en
    print(f"{(en-st)/1e3:7.1f} {g:6.1f}  {nm(r)[:40]:40s} grid {r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']} wg {r['Workgroup_Size_X']} lds {r['LDS_Block_Size']}")
