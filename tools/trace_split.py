import csv, statistics as st, sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
prev=None; a={}
for r in rows:
    n=r['Kernel_Name'].split('(')[0].split('<')[0].replace('void ','')
    d=int(r['End_Timestamp'])-int(r['Start_Timestamp'])
    key=(n, prev)
    a.setdefault(key,[]).append(d)
    prev=n
for k,v in sorted(a.items(), key=lambda x:-len(x[1])):
    if len(v)>5: print(k, len(v), 'dur med', st.median(v), 'mean %.0f'%st.mean(v))
