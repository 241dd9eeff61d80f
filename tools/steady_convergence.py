"""CPU model of the DNS covariance recursion on the config-2 batch (bench.py make_workload(2)): the
collapsed form's P ↦ Φ P(P + R)⁻¹R Φ' + Q (data-independent for fixed loadings) from the Lyapunov start,
and the step at which each candidate meets the kernel's freeze test (relative change ≤ 2^-46 and
estimated remaining drift d·ρ/(1 − ρ) ≤ 2^-50; yfm_fixedz.hpp FixedZFilter::freeze_test), per candidate
and per wave of 64.  numpy FP64, so the steps can differ from the kernel's by one.

    python tools/steady_convergence.py
"""
import sys, numpy as np
sys.path[:0]=['.','yieldfactormodels.jl_amd']
from yfm_amd import synthetic as S, KIND_DNS
from yfm_amd import params as PR
mats=S.maturities_30(); B=65536; T=600
Th=S.theta_batch(KIND_DNS,B,seed=S.BATCH_SEED)
Thc=np.stack([PR.transform_params(KIND_DNS,Th[:,b]) for b in range(B)],1)
# layout DNS: [gamma, sigma2, U (6: by column upper), delta(3), Phi(9 row-major)]
g=Thc[0]; s2=Thc[1]; Ucol=Thc[2:8]; dl=Thc[8:11]; Phi=Thc[11:20].T.reshape(B,3,3)
U=np.zeros((B,3,3)); k=0
for j in range(3):
    for i in range(j+1):
        U[:,i,j]=Ucol[k]; k+=1
Q=np.einsum('bli,blj->bij',U,U)
lam=(0.01+np.exp(Th[0]))[:,None]  # gamma unconstrained is theta[0] identity
tau=lam*mats[None]; e=np.exp(-tau); sl=(1-e)/tau
Z=np.stack([np.ones_like(sl),sl,sl-e],2)  # B,N,3
G=np.einsum('bni,bnj->bij',Z,Z); R=s2[:,None,None]*np.linalg.inv(G)
# P0: Lyapunov solve P = Phi P Phi' + Q via Kronecker
I9=np.eye(9)
K=I9[None]-np.einsum('bij,bkl->bikjl',Phi,Phi).reshape(B,9,9)
P=np.linalg.solve(K,Q.reshape(B,9,1)).reshape(B,3,3)
ok=np.all(np.isfinite(P),axis=(1,2))
conv=np.full(B,T,int); prevd=np.full(B,np.inf)
for t in range(T-1):
    Sm=P+R
    Pu=P@np.linalg.solve(Sm,R)
    Pn=Phi@Pu@np.transpose(Phi,(0,2,1))+Q
    Pn=0.5*(Pn+np.transpose(Pn,(0,2,1)))
    d=np.max(np.abs(Pn-P),axis=(1,2))/np.maximum(np.max(np.abs(Pn),axis=(1,2)),1e-300)
    rho=d/np.maximum(prevd,1e-300)
    # converged: the remaining drift d·rho/(1-rho) below 2^-50 relative
    drift=np.where(rho<0.999, d*rho/np.maximum(1-rho,1e-3), np.inf)
    newc=(conv==T)&(d<=2.0**-46)&(drift<=2.0**-50)
    conv[newc]=t+1
    prevd=d; P=Pn
conv[~ok]=0
print('lanes converged by step: quantiles', np.quantile(conv,[0.5,0.9,0.99,0.999,1.0]))
w=conv.reshape(-1,64).max(1)
print('waves: switch step quantiles', np.quantile(w,[0.1,0.5,0.9,1.0]), ' fraction of wave-steps in fast mode', np.mean((T-1-np.minimum(w,T-1))/(T-1)))
