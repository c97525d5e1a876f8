"""Per-prove kernel durations of mlh_sumcheck_prove_eq from a rocprofv3 kernel trace (dev tool):
setup, corner sums, head, 6-level fold, fold + tail corner sums, tail (usage: sc_split.py run_kernel_trace.csv)."""
import csv, sys, statistics as st
r=list(csv.DictReader(open(sys.argv[1])))
r.sort(key=lambda x:int(x['Start_Timestamp']))
idx=[i for i,x in enumerate(r) if 'eq_setup' in x['Kernel_Name'] and 'corner_sums' in r[i+1]['Kernel_Name'] and 'eq_tail' in r[i+2]['Kernel_Name']]
d=lambda x:(int(x['End_Timestamp'])-int(x['Start_Timestamp']))/1e3
names=['setup','corner','head','fold6','fold6xc','tail']
vals={n:[] for n in names}
span=[]
for i in idx:
    for k,n in enumerate(names): vals[n].append(d(r[i+k]))
    span.append((int(r[i+5]['End_Timestamp'])-int(r[i]['Start_Timestamp']))/1e3)
for n in names: print("%-8s mean %.2f min %.2f (n=%d)"%(n,st.mean(vals[n]),min(vals[n]),len(vals[n])))
print("device span setup..tail mean %.1f min %.1f"%(st.mean(span),min(span)))
