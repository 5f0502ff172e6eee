import sys, numpy as np, torch
sys.path.insert(0,'.'); sys.path.insert(0,'oracle')
import pkgload, vbhem_oracle as vo
vb = pkgload.load()
from vbhem_amd.estep import EStepEngine
dev = torch.device('cuda',0)
for name, N, ragged in [('C2',100,False),('C3',64,False),('C3',64,True),('C4',40,False),('C4',40,True),('C5',3,False)]:
    base, post, opt = vb.synth_workload(name, N=N, ragged=ragged)
    consts = vb.host.cluster_constants(post, base.covmode)
    eng = EStepEngine(base, post.K, post.S, opt['tau'], device=dev)
    eng.set_clusters(consts)
    out = eng.pairs(); torch.cuda.synchronize()
    ref = vo.c_estep_pairs(base.numpy(), consts, opt['tau'])
    errs = {k: float(np.max(np.abs(out[k].cpu().numpy()-ref[k]))/max(1e-300,np.max(np.abs(ref[k])))) for k in ref}
    print(name, N, 'ragged' if ragged else '', {k: f"{v:.1e}" for k,v in errs.items()}, 'fallback', eng.fallback_count(), flush=True)
