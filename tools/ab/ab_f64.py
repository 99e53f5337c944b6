import ctypes, os, sys
import numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import ivclab_amd._native as N, bench
N.load_library()
libs=[]
for p in sys.argv[1:]:
    L=ctypes.CDLL(os.path.abspath(p))
    for name,(a,r) in N._SIGS.items():
        fn=getattr(L,name,None)
        if fn is not None: fn.argtypes, fn.restype = a, r
    libs.append((p,L))
dev=torch.device("cuda:0")
seq=bench.inter_frames(60,1080,1920,seed=4,dev=dev)
y=bench.luma_f64(seq).contiguous()
mvs=[torch.empty((59,135,240),dtype=torch.int64,device=dev) for _ in libs]
st=torch.cuda.current_stream().cuda_stream
res={p:[] for p,_ in libs}
for rnd in range(4):
    for (p,L),mv in zip(libs,mvs):
        s,e=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
        f=lambda: N.check(L.ivc_motion_estimate_dev(y[:-1].data_ptr(), y[1:].data_ptr(), 10, 59, 1080, 1920, 16, 0, mv.data_ptr(), st))
        f(); s.record(); f(); f(); e.record(); torch.cuda.synchronize()
        res[p].append(s.elapsed_time(e)/2)
for (p,_),mv in zip(libs,mvs):
    print(p, "median %.3f ms"%np.median(res[p]), "same", bool(torch.equal(mv,mvs[0])))
