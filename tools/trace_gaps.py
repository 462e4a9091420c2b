"""Device idle time per call from a rocprofv3 kernel trace (kernel_trace.csv):
calls cut at each k_reset; for each call its span (k_reset to the next
k_reset), the time some kernel ran (union over queues), the idle time after
its last kernel, and every idle gap over 3 us with the kernel that ended it.

  python tools/trace_gaps.py TRACE.csv
"""
import csv,sys
kr=list(csv.DictReader(open(sys.argv[1])))
kr.sort(key=lambda r:int(r['Start_Timestamp']))
sh=lambda n:n.split('(')[0].replace('pmmg::','').replace('void ','')[:22]
idx=[i for i,r in enumerate(kr) if sh(r['Kernel_Name'])=='k_reset']
for c in range(len(idx)-1):
    seg=kr[idx[c]:idx[c+1]]
    t0=int(seg[0]['Start_Timestamp']); tn=int(kr[idx[c+1]]['Start_Timestamp'])
    iv=sorted((int(r['Start_Timestamp']),int(r['End_Timestamp'])) for r in seg)
    busy=0; cur_s,cur_e=iv[0]; gaps=[]
    for s,e in iv[1:]:
        if s>cur_e: busy+=cur_e-cur_s; gaps.append((s-cur_e, sh([r for r in seg if int(r['Start_Timestamp'])==s][0]['Kernel_Name']))); cur_s,cur_e=s,e
        else: cur_e=max(cur_e,e)
    busy+=cur_e-cur_s
    big=[(round(g/1e3,1),n) for g,n in gaps if g>3000]
    print(f'call {c}: span {(tn-t0)/1e3:7.1f} busy {busy/1e3:7.1f} idle-to-next {(tn-cur_e)/1e3:6.1f}  gaps>3us {big}')
