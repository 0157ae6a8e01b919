"""LDS bank model of the 4x2 kernel's split FIR (qpsk_rx.hip fir_split).

ds_read_b64 serves lanes 0-31 and 32-63 apart; float2 index f sits in bank
pair f mod 32; a group costs its largest number of distinct addresses in one
pair (MI355X_MICROARCH.md "LDS").  For every rx_timing rt in [3, 255] it counts
the extra LDS cycles per channel of pass 1 (59 loads: lanes 0..62 at M[15l +
rt + s], lane 63 on its F triple) and pass 2 (49 loads: one F output per lane)
under the round-5 mapping ("old": lane 63 on F[56], pass 2 j = l + (l >= 56) +
(l >= 60)), the rt-dependent lane-63 triple with a monotone pass 2 ("new") and
the kernel's table (kSplitTab: "tab").  Checks that every mapping computes
each of F[0..66] once.
    python3 profiles/probe/fir_split_banks.py
"""
kM1=1240
def cost(addrs):  # addrs: list of 64 float2 indices or None
    tot=0
    for g in (range(0,32),range(32,64)):
        cnt={}
        for l in g:
            a=addrs[l]
            if a is None: continue
            cnt.setdefault(a%32,set()).add(a)
        tot+=max([len(v) for v in cnt.values()] or [0])
    return tot
def old(rt):
    p1=[15*l+rt if l<63 else kM1+56 for l in range(64)]
    j=[l+(l>=56)+(l>=60) for l in range(64)]
    p2=[kM1+x for x in j]
    return p1,p2,{56,61,66},j
def new(rt):
    r=(rt+25)&31
    j0=r+32 if r<=24 else r
    holes={j0,j0+5,j0+10}
    p1=[15*l+rt if l<63 else kM1+j0 for l in range(64)]
    if r<=24:
        vals=[v for v in range(67) if v not in holes]
        j=vals
    else:
        B=[ (v-32 if v in holes else v) for v in range(35,67)]
        A=[v for v in range(67) if v not in holes and v not in B]
        assert len(A)==32, (r,len(A))
        j=A+B
    p2=[kM1+x for x in j]
    return p1,p2,holes,j
for name,f in (("old",old),("new",new)):
    t1=t2=0
    for rt in range(3,256):
        p1,p2,holes,j=f(rt)
        assert sorted(set(j)|holes)==list(range(67)) and len(set(j))==64 and not (set(j)&holes),(name,rt)
        t1+=sum(cost([a+s for a in p1]) for s in range(59))-2*59
        t2+=sum(cost([a+s for a in p2]) for s in range(49))-2*49
    n=253
    print(name,"extra cycles/channel pass1 %.1f pass2 %.1f"%(t1/n,t2/n))
def tab(r):
    j1=r+32 if r<=24 else r
    hole=lambda v: v in (j1,j1+5,j1+10)
    B=[]
    for i in range(32):
        v=35+i
        if hole(v): v-=32
        B.append(v)
    A=[v for v in range(67) if not hole(v) and v not in B]
    assert len(A)==32
    return j1,A+B
def new2(rt):
    r=(945+rt-kM1)&31
    j1,j=tab(r)
    p1=[15*l+rt if l<63 else kM1+j1 for l in range(64)]
    return p1,[kM1+x for x in j],{j1,j1+5,j1+10},j
t1=t2=0
for rt in range(3,256):
    p1,p2,holes,j=new2(rt)
    assert sorted(set(j)|holes)==list(range(67)) and len(set(j))==64 and not (set(j)&holes)
    t1+=sum(cost([a+s for a in p1]) for s in range(59))-2*59
    t2+=sum(cost([a+s for a in p2]) for s in range(49))-2*49
print("tab", t1/253, t2/253)
