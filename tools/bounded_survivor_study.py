"""Oracle study of the bounded exit's survivors (DESIGN.md "a mode-4 probe"):
the stage-0 fit and the 6/3/1 probes modelled with the oracle on G1 block rows,
then the exact search's MSE and winning modes over the blocks they leave, and
which extra probe (mode, shake ranks) would finish them.

    python tools/bounded_survivor_study.py
"""
import sys, numpy as np
import os; R=os.path.join(os.path.dirname(os.path.abspath(__file__)),'..'); sys.path.insert(0,os.path.join(R,'tests')); sys.path.insert(0,R)
import oracle_lib
from gfx_imagecompress_amd import synth
from test_gpu_bc7 import _block_mse, _src_blocks
MSE=0.5
def model(img):
    sb=_src_blocks(img)
    fit,_=oracle_lib.bc7_fit6_blocks(sb)
    done=_block_mse(fit,sb)<=MSE
    for mode in (6,3,1):
        oracle_lib.lib().orc_bc7_set_probe_init(int(mode==6))
        try:
            idx=np.where(~done)[0]
            if len(idx)==0: break
            cand=oracle_lib.bc7_blocks_ex(sb[idx], mode_mask=1<<mode, colour_restrict=False, shake_ranks=2)
        finally:
            oracle_lib.lib().orc_bc7_set_probe_init(0)
        ok=_block_mse(cand,sb[idx])<=MSE
        done[idx[ok]]=True
    return sb, done
g=synth.g1(8192,8192)
for name,img in (("top",g[0:16,0:2048]),("mid",g[4096:4112,0:2048]),("bottom",g[8176:8192,0:2048])):
    img=np.ascontiguousarray(img)
    sb,done=model(img)
    surv=np.where(~done)[0]
    print(name, len(sb), "survivors", len(surv), flush=True)
    if len(surv):
        ex=oracle_lib.bc7_blocks_ex(sb[surv])
        m=_block_mse(ex,sb[surv])
        modes=np.bincount(np.log2((ex[:,0].astype(int)&-ex[:,0].astype(int))).astype(int),minlength=8)
        print("  exact MSE of survivors: <=0.5:", (m<=0.5).mean(), "mean", m.mean(), "modes", modes)
print("--- extra probes on top+bottom survivors")
for name,img in (("top",g[0:16,0:2048]),("bottom",g[8176:8192,0:2048])):
    img=np.ascontiguousarray(img)
    sb,done=model(img)
    surv=np.where(~done)[0]; s=sb[surv]
    for label,mask,ranks in (("mode4 r2",1<<4,2),("mode5 r2",1<<5,2),("mode3 r8",1<<3,8),("mode1 r8",1<<1,8),("mode0 r2",1<<0,2),("mode2 r2",1<<2,2),("modes 1+3+4 r2",(1<<1)|(1<<3)|(1<<4),2)):
        c=oracle_lib.bc7_blocks_ex(s, mode_mask=mask, colour_restrict=False, shake_ranks=ranks)
        print(name,label,"catches",round((_block_mse(c,s)<=0.5).mean(),3),flush=True)
