"""One training step of a rocprofv3 --kernel-trace CSV (steps delimited by the RMSprop launches): span, GPU-busy time,
time at each stream concurrency, kernel time per queue and per kernel family, and the largest idle gaps.
Usage: python tools/step_overlap.py <run_kernel_trace.csv>"""
import csv, sys
from collections import defaultdict
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
# step boundaries: rmsprop_kernel dispatches (one or more per step); take the last rmsprop of each cluster
rms=[i for i,r in enumerate(rows) if 'rmsprop' in r['Kernel_Name']]
# cluster
ends=[]
for i in rms:
    if not ends or int(rows[i]['Start_Timestamp'])-int(rows[ends[-1]]['End_Timestamp'])>1e6: ends.append(i)
    else: ends[-1]=i
print('steps found', len(ends))
# analyze the window between ends[-3] and ends[-2]
a,b=ends[-3]+1, ends[-2]+1
win=rows[a:b]
t0=int(win[0]['Start_Timestamp']); t1=max(int(r['End_Timestamp']) for r in win)
print('step span ms', (t1-t0)/1e6, 'dispatches', len(win))
# busy union and concurrency
ev=[]
for r in win:
    ev.append((int(r['Start_Timestamp']),1)); ev.append((int(r['End_Timestamp']),-1))
ev.sort()
cur=0; last=t0; busy=0; conc=defaultdict(int)
for t,d in ev:
    if cur>0: busy+=t-last
    conc[cur]+=t-last
    cur+=d; last=t
print('busy ms', busy/1e6, 'conc', {k:round(v/1e6,3) for k,v in sorted(conc.items())})
streams=defaultdict(float)
for r in win: streams[r['Queue_Id']]+= (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6
print('per queue kernel ms', dict(streams))
# categories
def cat(n):
    for k,c in [('conv_bf3','vgg conv_bf3'),('vgg_conv0','vgg conv0'),('gram','gram'),('maxpool','pool'),('wgrad9','wgrad9'),('wgrad_x6','wgrad_x6'),('wgradT9','wgradT9'),('wgrad','wgrad other'),('wino9','start conv fwd'),('wino_x6','wino_x6'),('conv_lite','conv_lite'),('last','last'),('norm_bwd','norm bwd'),('bn_','bn'),('pw_','pw'),('dw_','dw'),('se_','se'),('stem','stem'),('conv_mfma','conv_mfma'),('slab','slab'),('head','head'),('rowdot','se/head'),('outer','se/head'),('tap3','tap3'),('fill','fill'),('copy','copy')]:
        if k in n: return c
    return 'other'
agg=defaultdict(lambda:[0,0.0])
for r in win:
    c=cat(r['Kernel_Name']); agg[c][0]+=1; agg[c][1]+=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6
for k,v in sorted(agg.items(), key=lambda x:-x[1][1]): print(f"{k:16s} {v[0]:4d} {v[1]:7.3f} ms")
# gaps: time where nothing runs, list biggest
gaps=[]
last_end=t0
for r in win:
    s=int(r['Start_Timestamp'])
    if s>last_end: gaps.append((s-last_end, r['Kernel_Name'][:60]))
    last_end=max(last_end,int(r['End_Timestamp']))
gaps.sort(reverse=True)
print('idle total ms', sum(g for g,_ in gaps)/1e6, 'top gaps', [(round(g/1e3,1),n) for g,n in gaps[:8]])
