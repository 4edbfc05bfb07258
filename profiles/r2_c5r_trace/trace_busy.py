import csv,sys,collections
d=sys.argv[1]
cp=list(csv.DictReader(open(d+'/run_memory_copy_trace.csv')))
kt=list(csv.DictReader(open(d+'/run_kernel_trace.csv')))
# focus on the timed region: last ~N H2D bytes; use the big H2D copies (>1MB) after the warmup
def iv(r): return int(r['Start_Timestamp']), int(r['End_Timestamp'])
h2d=[iv(r) for r in cp if r['Direction'].endswith('HOST_TO_DEVICE')]
d2h=[iv(r) for r in cp if r['Direction'].endswith('DEVICE_TO_HOST')]
import re
ks=[(iv(r), re.search(r'(\w+_kernel|copyBuffer)', r['Kernel_Name']).group(1)) for r in kt]
# timed region: from the first kernel of the last 70% of sha launches to end
sha=[k for k in ks if 'sha256' in k[1]]
t0=sha[len(sha)//4][0][0]; t1=max(e for (s,e),_ in ks)
def busy(iv_list, a, b):
    xs=sorted((max(s,a),min(e,b)) for s,e in iv_list if e>a and s<b)
    tot=0; cur=None
    for s,e in xs:
        if cur is None or s>cur[1]:
            if cur: tot+=cur[1]-cur[0]
            cur=[s,e]
        else: cur[1]=max(cur[1],e)
    if cur: tot+=cur[1]-cur[0]
    return tot
W=t1-t0
print(d, 'window ms', W/1e6)
print(' H2D busy %.1f%%  D2H busy %.1f%%'%(100*busy(h2d,t0,t1)/W, 100*busy(d2h,t0,t1)/W))
n_h2d=sum(1 for s,e in h2d if s>=t0 and e<=t1); n_d2h=sum(1 for s,e in d2h if s>=t0 and e<=t1)
print(' copies in window: h2d',n_h2d,'d2h',n_d2h)
byk=collections.defaultdict(list)
for (s,e),n in ks:
    if s>=t0: byk[n].append((e-s)/1e6)
for n,v in byk.items(): print('  %-28s n=%d avg %.2f ms max %.2f'%(n,len(v),sum(v)/len(v),max(v)))
# H2D gaps: idle periods longer than 0.1ms
xs=sorted((s,e) for s,e in h2d if e>t0 and s<t1)
gaps=[]; end=xs[0][1]
for s,e in xs[1:]:
    if s>end: gaps.append(s-end)
    end=max(end,e)
print(' H2D idle gaps >0.1ms: n=%d total %.1f ms'%(sum(1 for g in gaps if g>1e5), sum(g for g in gaps if g>1e5)/1e6))
# biggest H2D copy durations & rates
big=[(e-s) for s,e in h2d if s>=t0 and e<=t1]
