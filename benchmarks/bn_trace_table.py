import csv, sys, glob, os
SH=[(64,112,False,True),(64,56,False,True),(256,56,True,True),(256,56,False,False),(128,56,False,True),(128,28,False,True),(512,28,True,True),(512,28,False,False),(256,28,False,True),(256,14,False,True),(1024,14,True,True),(1024,14,False,False),(512,14,False,True),(512,7,False,True),(2048,7,True,True),(2048,7,False,False)]
def load(path):
    rows=list(csv.DictReader(open(path)))
    rows.sort(key=lambda r:int(r['Start_Timestamp']))
    def durs(sub, per):
        d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in rows if sub in r['Kernel_Name']]
        return [sorted(d[i*per:(i+1)*per])[per//2] for i in range(len(d)//per)]
    return {k:durs(*v) for k,v in {'stats':('bn_stats',10),'fin_f':('bn_fwd_finalize',10),'apply':('bn_apply_kernel',10),'bwdred':('bn_bwd_reduce',8),'fin_b':('bn_bwd_finalize',8),'bapply':('bn_bwd_apply',8)}.items()}
counts={1:1,2:6,3:3,4:1,5:1,6:7,7:4,8:1,9:1,10:11,11:6,12:1,13:1,14:5,15:3,16:1}
files=sorted(glob.glob(sys.argv[1] if len(sys.argv)>1 else '/root/repo/gpurun_out/bnt/trace_*.csv'))
res={os.path.basename(f)[6:-4][:40]:load(f) for f in files}
keys=list(res)
print('shape'.ljust(12), '  '.join(f"{k:>18s}" for k in keys))
for i,(C,H,_,_) in enumerate(SH):
    print(f"C{C}H{H}".ljust(12), '  '.join(f"{res[k]['stats'][i]:7.1f}/{res[k]['bwdred'][i]:7.1f}" for k in keys))
for k in keys:
    tot=sum(counts[i+1]*(res[k]['stats'][i]+res[k]['bwdred'][i]+res[k]['fin_f'][i]+res[k]['fin_b'][i]) for i in range(16))
    app=sum(counts[i+1]*(res[k]['apply'][i]+res[k]['bapply'][i]) for i in range(16))
    print(k, 'per-step stats+bwdred+finalize (ResNet-50 counts):', round(tot/1e3,3),'ms; apply+bwd-apply:', round(app/1e3,3), 'ms')
