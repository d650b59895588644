"""Model of the fit's memory-bound skip on C4: the streamed node groups of
8 (node order), each group's smallest U = floor(fc / P) and V = floor(fm / P), and the
(group, 64-spec wave) pairs that could skip the memory quotient (m_max <= V_min), the CPU
quotient (c_max <= U_min) or both, for several spec orders; prints the average VALU per node
x wave (3 full, 2.5 CPU known, 2 memory known, 0.125 both).

  python scripts/probe/mskip_model.py
"""
import numpy as np, sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from kubernetesclustercapacity_amd import synth
c = synth.config_cluster("C4", limits=False)
sc, sm = synth.config_specs("C4")
cs = np.zeros(c.n_containers+1, np.uint64); np.cumsum(c.cpu_req, out=cs[1:]); uc = cs[c.node_ptr[1:]]-cs[c.node_ptr[:-1]]
ms = np.zeros(c.n_containers+1, np.uint64); np.cumsum(c.mem_req.view(np.uint64), out=ms[1:]); um = (ms[c.node_ptr[1:]]-ms[c.node_ptr[:-1]]).view(np.int64)
fc = np.where(c.alloc_cpu > uc, c.alloc_cpu - uc, 0).astype(np.int64)
fm = np.where(c.alloc_mem > um, c.alloc_mem - um, 0)
P = c.alloc_pods
st = (fc>0)&(fm>0)&(P>=1)&(fc < 2**23)&(fm < 2**50)
fc, fm, P = fc[st], fm[st], P[st]
n = fc.size; ng = n//8
U = (fc//P)[:ng*8].reshape(ng,8).min(1); V = (fm//P)[:ng*8].reshape(ng,8).min(1)
print("streamed", n, "groups", ng)
c_s = sc.astype(np.int64); m_s = sm
def cost(order):
    cw = c_s[order].reshape(-1,64); mw = m_s[order].reshape(-1,64)
    cmax = cw.max(1); mmax = mw.max(1)
    tot=0.0
    # per (group, wave)
    cok = U[:,None] >= cmax[None,:]
    mok = V[:,None] >= mmax[None,:]
    full = cok & mok
    conly = cok & ~mok
    monly = mok & ~cok
    none = ~cok & ~mok
    # VALU per node: none 3, c-known (skip pk_mul): 2.5, m-known (skip mul_f64): 2.0, full: 0.125
    v = (none*3 + conly*2.5 + monly*2.0 + full*0.125).mean()
    return v, full.mean(), conly.mean(), monly.mean()
S=sc.size
print("random order", cost(np.arange(S)))
print("sorted by m", cost(np.argsort(m_s, kind='stable')))
print("sorted by c", cost(np.argsort(c_s, kind='stable')))
# 2D: 8 m-blocks of 512, within by c
om = np.argsort(m_s, kind='stable')
for nbk in (4, 8, 16, 32, 64):
    blk = S//nbk
    o2 = np.concatenate([om[i*blk:(i+1)*blk][np.argsort(c_s[om[i*blk:(i+1)*blk]], kind='stable')] for i in range(nbk)])
    print("2D m-blocks", nbk, cost(o2))
