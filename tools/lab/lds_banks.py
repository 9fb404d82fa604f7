import itertools
G128=[[0,1,2,3,12,13,14,15,20,21,22,23,24,25,26,27],[4,5,6,7,8,9,10,11,16,17,18,19,28,29,30,31]]
G128=G128+[[l+32 for l in g] for g in G128]
def cyc_read128(addrs):  # addrs: float index per lane (16B aligned); bank mod 64, 4 banks per lane
    tot=0
    for g in G128:
        banks={}
        for l in g:
            a=addrs[l]
            for b in range(4):
                bk=(a+b)%64; banks.setdefault(bk,set()).add(a+b)
        tot+=max(len(v) for v in banks.values())
    return tot  # 4 = conflict-free
def cyc_write128(addrs):  # 8 groups of 8 contiguous lanes, bank mod 32
    tot=0
    for g0 in range(0,64,8):
        banks={}
        for l in range(g0,g0+8):
            a=addrs[l]
            for b in range(4):
                bk=(a+b)%32; banks.setdefault(bk,set()).add(a+b)
        tot+=max(len(v) for v in banks.values())
    return tot  # 8
def cyc_read32(addrs):
    tot=0
    for g0 in (0,32):
        banks={}
        for l in range(g0,g0+32):
            a=addrs[l]; banks.setdefault(a%32,set()).add(a)
        tot+=max(len(v) for v in banks.values())
    return tot  # 2
def lanes():
    for l in range(64): yield l, l&15, l>>4, l//16, l%16
def eval_S(S):
    c={}
    c['w_tile']=max(cyc_write128([ (4*k+l//16)*S + 4*(l%16) for l in range(64)]) for k in range(4))
    c['dW_r32']=max(cyc_read32([ (4*(l>>4)+kk)*S + 16*ni + (l&15) for l in range(64)]) for kk in range(4) for ni in range(4))
    c['dx_r128']=max(cyc_read128([ (l&15)*S + 32*s2 + 8*(l>>4) + h*4 for l in range(64)]) for s2 in range(2) for h in range(2))
    c['mask_r128']=max(cyc_read128([ (l&15)*S + 16*mt + 4*(l>>4) for l in range(64)]) for mt in range(4))
    c['dxw_w128']=max(cyc_write128([ (l&15)*S + 16*mt + 4*(l>>4) for l in range(64)]) for mt in range(4))
    c['vk_r128']=max(cyc_read128([ (4*k+l//16)*S + 4*(l%16) for l in range(64)]) for k in range(4))
    return c
def eval_SB(SB):  # halves
    return max(cyc_read128([ ((16*mt+(l&15))*SB + 32*s2 + 8*(l>>4))//2 for l in range(64)]) for mt in range(4) for s2 in range(2))
print('S=68', eval_S(68))
best=[]
for S in range(64,160,4):
    c=eval_S(S); ideal={'w_tile':8,'dW_r32':2,'dx_r128':4,'mask_r128':4,'dxw_w128':8,'vk_r128':4}
    extra=sum(c[k]-ideal[k] for k in c)
    best.append((extra,S,c))
best.sort()
for b in best[:6]: print(b)
print('SB=72', eval_SB(72))
for SB in range(64,200,8): print(SB, eval_SB(SB), end='; ')

print()
def eval_f(S, f):
    A=lambda r,c: r*S + c + 4*f(r)
    c={}
    c['w_tile']=max(cyc_write128([ A(4*k+l//16, 4*(l%16)) for l in range(64)]) for k in range(4))
    c['dW_r32']=max(cyc_read32([ A(4*(l>>4)+kk, 16*ni + (l&15)) for l in range(64)]) for kk in range(4) for ni in range(4))
    c['dx_r128']=max(cyc_read128([ A(l&15, 32*s2 + 8*(l>>4) + h*4) for l in range(64)]) for s2 in range(2) for h in range(2))
    c['mask_r128']=max(cyc_read128([ A(l&15, 16*mt + 4*(l>>4)) for l in range(64)]) for mt in range(4))
    c['dxw_w128']=max(cyc_write128([ A(l&15, 16*mt + 4*(l>>4)) for l in range(64)]) for mt in range(4))
    c['vk_r128']=max(cyc_read128([ A(4*k+l//16, 4*(l%16)) for l in range(64)]) for k in range(4))
    return c
ideal={'w_tile':8,'dW_r32':2,'dx_r128':4,'mask_r128':4,'dxw_w128':8,'vk_r128':4}
res=[]
for S in range(64,100,4):
  for a in range(0,4):
    for b in range(0,16):
      f=lambda r,a=a,b=b: ((r>>a)*b)%16
      c=eval_f(S,f); ex=sum(c[k]-ideal[k] for k in c)
      res.append((ex,S,a,b,c))
res.sort(key=lambda x:(x[0],x[1]))
for r in res[:8]: print(r)
