import csv,glob,sys
for d in sys.argv[1:]:
    f=glob.glob(d+"/**/run_kernel_trace.csv",recursive=True)[0]
    rows=sorted(csv.DictReader(open(f)),key=lambda r:int(r["Start_Timestamp"]))
    prev=None; out=[]
    for r in rows:
        s=int(r["Start_Timestamp"]);e=int(r["End_Timestamp"]); n=r["Kernel_Name"]
        tag='S' if 'true' in n else ('P' if 'leapfrog' in n else ('R' if 'reduce' in n else ('C' if 'opy' in n else ('F' if 'ill' in n else n[:12]))))
        out.append(f"{tag}{(e-s)/1e3:.0f}/{(s-prev)/1e3 if prev else 0:.0f}"); prev=e
    print(d); print(' '.join(out[-40:]))
