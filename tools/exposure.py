#!/usr/bin/env python3
"""Exposure of one steady-state prove period of a rocprofv3 kernel trace (tools/gpu_trace.sh):
the period between the 2nd and 3rd k_p2_quotient launches (one prove), the time k_piece_sum* is
active, and the time each other kernel runs while no piece sum does.

usage: python tools/exposure.py <kernel_trace.csv>
"""
import csv,collections,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r['s']=int(r['Start_Timestamp']); r['e']=int(r['End_Timestamp'])
    r['n']=r['Kernel_Name'].replace("(anonymous namespace)::","").split("(")[0].replace("void ","").replace("eon::","")
q=sorted([r for r in rows if 'k_p2_quotient' in r['n']],key=lambda r:r['s'])
a,b=q[1]['s'],q[2]['s']
win=[dict(r) for r in rows if r['e']>a and r['s']<b]
for r in win: r['s']=max(r['s'],a); r['e']=min(r['e'],b)
ev=sorted([(r['s'],1,r['n']) for r in win]+[(r['e'],-1,r['n']) for r in win])
active=collections.Counter(); last=a; idle=0; crit=0; exp=collections.defaultdict(float)
busy=collections.defaultdict(float)
for t,d,n in ev:
    dt=(t-last)/1e6
    if dt>0:
        names=[k for k,v in active.items() if v>0]
        if not names: idle+=dt
        elif any('k_piece_sum' in k for k in names): crit+=dt
        else:
            for k in names: exp[k]+=dt/len(names)
    active[n]+=d; last=t
print('period %.1f ms: piece active %.1f, idle %.1f, exposed %.1f'%((b-a)/1e6,crit,idle,sum(exp.values())))
for k,v in sorted(exp.items(),key=lambda kv:-kv[1])[:25]: print('  %-45s %7.2f'%(k[:45],v))
