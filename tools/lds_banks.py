#!/usr/bin/env python3
"""Exhaustive LDS bank-conflict count of spec3.h exchange layouts (MI355X_MICROARCH.md LDS table:
ds_write_b64 in 4 groups of 16 lanes over 32 banks, ds_read_b64 in 2 groups of 32 lanes over 64
banks).  Prints the extra LDS cycles per pass for each pad of exchange B: pad 11 is the only
small pad with zero on both of its accesses (exchange A keeps the identity layout)."""
import itertools
M=18750; R1,R2,R3=25,30,25; NB1,NB2,NB3=M//R1,M//R2,M//R3
def phys(x,PAD,S=750): return x + (x//S)*PAD
def cost(addrs, write):
    # addrs: list of (lane, float2 index) active lanes; returns extra cycles
    g = 16 if write else 32; nb = 32 if write else 64
    extra=0
    groups={}
    for l,a in addrs: groups.setdefault(l//g,[]).append(a)
    for gl in groups.values():
        banks={}
        for a in set(gl):
            for d in (2*a, 2*a+1):
                banks.setdefault(d%nb,set()).add(a)
        extra += max(len(v) for v in banks.values())-1
    return extra
def evaluate(PAD, T=768):
    tot={}
    # pass1 writes x = j*R1 + r (j<NB1)
    c=0
    for r in range(R1):
        for w in range(0,T,64):
            c+=cost([(l, phys(j*R1+r,PAD)) for l in range(64) for j in [w+l] if j<NB1], True)
    tot['p1w']=c
    c=0
    for r in range(R2):
        for w in range(0,T,64):
            c+=cost([(l, phys(j+NB2*r,PAD)) for l in range(64) for j in [w+l] if j<NB2], False)
    tot['p2r']=c
    c=0
    for r in range(R2):
        for w in range(0,T,64):
            c+=cost([(l, phys((j//R1)*R1*R2 + j%R1 + R1*r,PAD)) for l in range(64) for j in [w+l] if j<NB2], True)
    tot['p2w']=c
    c=0
    for r in range(R3):
        for w in range(0,T,64):
            c+=cost([(l, phys(j+NB3*r,PAD)) for l in range(64) for j in [w+l] if j<NB3], False)
    tot['p3r']=c
    return tot
for PAD in [0,1,2,3,5,7,9,11,13,15,16,17,19,21,23,27,29,31,33]:
    t=evaluate(PAD); print(PAD, t, sum(t.values()))
