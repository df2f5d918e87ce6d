import re, sys
from collections import Counter
s=open(sys.argv[1]).read()
def cls(ins):
    op=ins.split()[0]
    if op.startswith('v_mfma'): return 'mfma'
    if op.startswith('v_'): return 'valu'
    if op.startswith('s_waitcnt'): return 'wait'
    if op.startswith('s_'): return 'salu'
    if op.startswith('ds_'): return 'lds'
    if op.startswith('buffer_') or op.startswith('global_'): return 'vmem'
    if op.startswith('scratch'): return 'scratch'
    return 'other'
for name in sys.argv[2:]:
    i=s.index(name+':'); j=s.index('.Lfunc_end', i)
    body=s[i:j].split('\n')
    blocks=[];cur=[];lab='entry'
    for l in body:
        if re.match(r'^\.LBB\d+_\d+:', l) or l.startswith('; %bb.'):
            blocks.append((lab,cur)); lab=l; cur=[]
        else:
            t=l.strip()
            if t and not t.startswith(';') and not t.startswith('.'): cur.append(t)
    blocks.append((lab,cur))
    tot=Counter(); allc=Counter()
    for lab,ins in blocks:
        c=Counter(cls(x) for x in ins); allc+=c
        if 'Depth=2' in lab or 'Depth=3' in lab: tot+=c
    print(name[30:80], 'loop', dict(tot), '| kernel', dict(allc))
