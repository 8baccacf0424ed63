"""Per-trial timeline of a rehearsal replay under rocprofv3 (tools/rehearse_ranks.sh with PROF=1):
for each trial, from the kernel trace -- the upload stream's plan and window kernels (stream 1,
starting at the trial's scatter_rows_kernel) and the blocking batch on the high-priority stream
(stream 2) -- the host's gap after the previous blocking batch, the upload span (plan part, window
part), the gap to the blocking batch and the blocking batch's span.
    python3 tools/trial_timeline.py <run_kernel_trace.csv>
"""
import csv, sys, statistics as st
f=sys.argv[1]
rows=[]
with open(f) as fh:
    for r in csv.DictReader(fh):
        rows.append((int(r['Start_Timestamp']),int(r['End_Timestamp']),r['Kernel_Name'],int(r['Stream_Id'])))
rows.sort()
# trials: a scatter_rows on stream 1 starts a trial's upload
tr=[]; cur=None
for s,e,n,sid in rows:
    if sid==1 and 'scatter_rows' in n:
        cur={'copy':s,'up':[],'blk':[],'fill':[]}; tr.append(cur)
    if cur is None: continue
    if sid==1: cur['up'].append((s,e,n))
    elif sid==2:
        (cur['fill'] if 'fillBuffer' in n else cur['blk']).append((s,e))
def q(v): v=sorted(v); return "p10 %.0f p50 %.0f p90 %.0f mean %.0f"%(v[len(v)//10],v[len(v)//2],v[9*len(v)//10],sum(v)/len(v))
A=[];U=[];G=[];S=[];F=[];T=[];W=[];P=[]
for i in range(1,len(tr)-1):
    t=tr[i]; p=tr[i-1]
    if not t['blk'] or not p['blk']: continue
    pend=max(e for s,e in p['blk'])
    upend=max(e for s,e,n in t['up'])
    plend=max([e for s,e,n in t['up'] if 'plan' in n or 'scatter' in n])
    bs=min(s for s,e in t['blk']); be=max(e for s,e in t['blk'])
    A.append((t['copy']-pend)/1e3); U.append((upend-t['copy'])/1e3); P.append((plend-t['copy'])/1e3); W.append((upend-plend)/1e3)
    G.append((bs-upend)/1e3); S.append((be-bs)/1e3); T.append((be-pend)/1e3)
    if t['fill']: F.append((bs-min(s for s,e in t['fill']))/1e3)
print("trials",len(A))
for name,v in (("prev blocking end -> copy start (host)",A),("upload span",U),(" plan part",P),(" window part",W),("upload end -> blocking start",G),("fill start -> blocking start",F),("blocking span",S),("trial (end to end)",T)):
    print("%-40s %s"%(name,q(v)))
# the upload stream's kernels: duration per launch and the gap before each (back-to-back launches
# of one stream show ~0 gap; a gap is the host issuing late)
import collections, re
dur = collections.defaultdict(list); gap = collections.defaultdict(list)
up = [(s, e, n) for s, e, n, sid in rows if sid == 1]
for i, (s, e, n) in enumerate(up):
    m = re.search(r'(\w+_kernel)', n); k = m.group(1) if m else n[:30]
    dur[k].append(e - s)
    if i: gap[k].append(s - up[i - 1][1])
for k in dur:
    d = sorted(dur[k]); g = sorted(gap[k]) or [0]
    print("%-26s n %7d  dur p50 %7.1f mean %7.1f us  gap before p50 %6.1f us" % (k, len(d), d[len(d) // 2] / 1e3, sum(d) / len(d) / 1e3, g[len(g) // 2] / 1e3))
