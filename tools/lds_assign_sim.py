"""orient_desc's sample reads: how much a static per-lane re-assignment of the lane's 4 tests to
the 4 descriptor words (any permutation, and either sample of a test first) could cut the bank
conflicts of its ds_read2_b32 gathers (MI355X_MICROARCH.md LDS table: per 32-lane group, bank =
dword mod 32, identical addresses broadcast -- approximated here without the broadcast). Coordinate
descent over the 384 options per lane on 120 random angles, scored on 300 others.
Result (profiles/r9j_lds_assign_sim.txt): 2.54 -> 2.18 extra cycles per 32-lane group and dword,
-14 % of the sample gathers' conflict cycles, before the SALU word reassembly and per-lane compare
selects such an assignment costs -- not built.
Usage: python tools/lds_assign_sim.py"""
import os
import re, numpy as np, itertools
ROOT=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
s=open(os.path.join(ROOT,'slam_framework_amd/csrc/orb_pattern.inc')).read(); s=re.sub(r"//.*","",s)
pat=np.array([int(x) for x in re.findall(r"-?\d+",s)][-1024:]).reshape(256,2,2)
stride=52
rng=np.random.default_rng(0)
def addr(ths):
    c,sn=np.cos(ths)[:,None,None],np.sin(ths)[:,None,None]
    x=np.rint(pat[None,...,0]*c-pat[None,...,1]*sn).astype(int)+18
    y=np.rint(pat[None,...,0]*sn+pat[None,...,1]*c).astype(int)+18
    return (x*stride+y)*2//4   # (n,256,2)
perms=list(itertools.permutations(range(4)))
opts=[(p,sw) for p in perms for sw in range(16)]
NO=len(opts)
# option table: slot -> (r_test, e_sample)
OT=np.array([[ (p[sl//2], (sl%2)^((sw>>(sl//2))&1)) for sl in range(8)] for (p,sw) in opts])  # (NO,8,2)
def slot_addr(A, L, oi):  # A (n,256,2) -> (n, len(oi), 8)
    r=OT[oi,:,0]; e=OT[oi,:,1]
    return A[:, 64*r+L, e]
def cost(A, assign):
    n=A.shape[0]
    D=np.stack([slot_addr(A,L,np.array([assign[L]]))[:,0] for L in range(64)],1)  # (n,64,8)
    tot=0
    for g in (slice(0,32),slice(32,64)):
        for k in range(4):
            banks=(D[:,g,:]+k)%32  # (n,32,8)
            cnt=np.zeros((n,8,32),int)
            for l in range(32): np.add.at(cnt,(np.arange(n)[:,None],np.arange(8)[None,:],banks[:,l,:]),1)
            tot+=(cnt.max(2)-1).sum()
    return tot/(n*2*8*4)
train=addr(rng.uniform(0,2*np.pi,120)); test=addr(rng.uniform(0,2*np.pi,300))
ident=[opts.index(((0,1,2,3),0))]*64
print("baseline train",cost(train,ident),"test",cost(test,ident),flush=True)
assign=list(ident)
nt=train.shape[0]
allD=np.stack([slot_addr(train,L,np.arange(NO)) for L in range(64)],1)  # (nt,64,NO,8)
for it in range(3):
    for L in rng.permutation(64):
        gl=range(0,32) if L<32 else range(32,64)
        # counts without lane L
        cnt=np.zeros((nt,8,4,32),int)
        for l in gl:
            if l==L: continue
            d=allD[:,l,assign[l],:]  # (nt,8)
            for k in range(4):
                np.add.at(cnt,(np.arange(nt)[:,None],np.arange(8)[None,:],k,(d+k)%32),1)
        M0=cnt.max(3)  # (nt,8,4)
        best=None
        dL=allD[:,L,:,:]  # (nt,NO,8)
        tot=np.zeros(NO)
        for k in range(4):
            b=(dL+k)%32
            c=np.take_along_axis(cnt[:,:,k,:][:,None,:,:].repeat(NO,1), b[...,None],3)[...,0]+1  # (nt,NO,8)
            tot+=np.maximum(M0[:,None,:,k],c).sum((0,2))
        assign[L]=int(np.argmin(tot))
    print("iter",it,"train",cost(train,assign),"test",cost(test,assign),flush=True)
