import sys, time, cProfile, pstats, numpy as np
sys.path.insert(0, '.')
import bench_grief as b, torch
import gp_grief_amd as gg, gp_grief_amd.grid, gp_grief_amd.kern, gp_grief_amd.models
gg.native.load()
d,m,kind,p,n,_=b.CONFIGS['C2']
x,y,xt=b.make_data(d,n)
for rep in range(3):
    mdl=b.build_model(gg,d,m,kind,p,x,y,0.01)
    torch.cuda.synchronize()
    pr=cProfile.Profile(); pr.enable()
    t=time.perf_counter(); mdl.kern._setup_inducing_cov(); torch.cuda.synchronize(); dt=time.perf_counter()-t
    pr.disable()
    print('setup', dt*1e3, 'ms')
pstats.Stats(pr).sort_stats('cumulative').print_stats(18)
from gp_grief_amd.tensors import device_sym_eig
for mm in (128, 200):
    F=[np.exp(-0.5*np.subtract.outer(np.linspace(0,1,mm),np.linspace(0,1,mm))**2/0.04)+1e-12*np.eye(mm) for _ in range(4)]
    device_sym_eig(F); torch.cuda.synchronize()
    t=time.perf_counter(); device_sym_eig(F); torch.cuda.synchronize(); print('eig 4 x', mm, (time.perf_counter()-t)*1e3,'ms')
