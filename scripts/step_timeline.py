"""Per-kernel microseconds of one step (between the last two k_classify_v4
launches) of a rocprofv3 kernel trace: python scripts/step_timeline.py run_kernel_trace.csv"""
import csv,sys,collections,re
rows=list(csv.DictReader(open(sys.argv[1])))
idx=[k for k,r in enumerate(rows) if 'k_classify_v4' in r['Kernel_Name']]
a,b=idx[-2],idx[-1]
seq=rows[a:b]
agg=collections.OrderedDict()
for r in seq:
    d=int(r['End_Timestamp'])-int(r['Start_Timestamp'])
    nm=r['Kernel_Name']
    m=re.search(r'(k_\w+|rocprim|fillBuffer|copyBuffer|at::native)',nm)
    n=m.group(1) if m else nm[:30]
    agg[n]=agg.get(n,0)+d
for k,v in agg.items(): print("%8.1f %s"%(v/1e3,k))
print("total", sum(agg.values())/1e3, "span", (int(seq[-1]['End_Timestamp'])-int(seq[0]['Start_Timestamp']))/1e3)
