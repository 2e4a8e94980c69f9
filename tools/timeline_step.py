import csv, glob, sys
rows=[]
for f in glob.glob(sys.argv[1]+'/**/*kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r['Start_Timestamp']),int(r['End_Timestamp']),r['Kernel_Name'][:60]))
rows.sort()
idx=[i for i,r in enumerate(rows) if 'k_compress<2' in r[2]]
i0=idx[-3]
prev=rows[i0-1][1]
for s,e,n in rows[i0-1:i0+8]:
    print(f"{(s-prev)/1e3:7.2f} gap  {(e-s)/1e3:7.2f} us  {n}"); prev=e
