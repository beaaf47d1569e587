#!/usr/bin/env python3
"""CPU simulation of the incremental region update of the W = 1 rule audit (RegionSet1 in
sparc-gym_amd/csrc/sparc_rules.hpp: ring_simple, remove / add / rebuild) against the full flood
of every region (SPaRC_Gym._compute_regions 422-454 as audit_r floods it), on random walks with
pops, resets and gaps over 5x5 and 7x7 lattices.  An algorithm check (the kernels' INC shapes
are tested against the default audit on the GPU, test_rule_rollout_shapes_equal_default); it
prints the count of rebuilds, simple removes, splits and adds.

    python tools/inc_regions_sim.py [boards]
"""
import random
import sys
def ring_simple(idx):
    order=[3,6,7,8,5,2,1,0]
    fg=next((k for k in range(8) if not (idx>>order[k])&1),-1)
    if fg<0: return 1
    runs=0; inn=False; h4=False
    for k in range(1,9):
        pos=(fg+k)&7; on=(idx>>order[pos])&1
        if on:
            if not inn: inn=True; h4=False
            h4 |= (pos&1)==0
        elif inn:
            inn=False; runs+= 1 if h4 else 0
    if inn: runs += 1 if h4 else 0
    return 1 if runs<=1 else 0
LUT=[ring_simple(i) for i in range(512)]
M=(1<<64)-1
def flood(seed,a,P):
    r=seed
    while True:
        up=((((a+r)&M)^a)&a)|r
        nx=(up|(r>>1)|((r<<P)&M)|(r>>P))&a
        if nx==r: return r
        r=nx
def ring_index(a,p,P):
    b=((a<<(P+1))&M)>>p
    return (b&7)|(((b>>P)&7)<<3)|(((b>>(2*P))&7)<<6)
def full(cells,a,P):
    rem=cells; out=[]
    while rem:
        R=flood(rem&-rem,a,P); out.append(R); rem&=~R
    return out
def run(seed):
    rnd=random.Random(seed)
    X=Y=rnd.choice([5,7]); P=Y+1
    lattice=0;cells=0
    for x in range(X):
        for y in range(Y):
            b=x*P+y
            if x%2==1 and y%2==1: cells|=1<<b
            else: lattice|=1<<b
    gaps=0
    for x in range(X):
        for y in range(Y):
            if (x+y)%2==1 and rnd.random()<0.15: gaps|=1<<(x*P+y)
    # path on vertices+edges: start at a random vertex
    pts=[(x,y) for x in range(0,X,2) for y in range(0,Y,2)]
    path=[rnd.choice(pts)]
    regs=None; vis=None; stats=[0,0,0,0]
    for t in range(200):
        if rnd.random()<0.25 and len(path)>1: path.pop()
        elif rnd.random()<0.05: path=[rnd.choice(pts)]
        else:
            x,y=path[-1]; dx,dy=rnd.choice([(1,0),(-1,0),(0,1),(0,-1)])
            nx,ny=x+dx,y+dy
            if 0<=nx<X and 0<=ny<Y and not(nx%2 and ny%2) and (nx,ny) not in path: path.append((nx,ny))
        v=0
        for (x,y) in path: v|=1<<(x*P+y)
        a=(lattice&~(gaps|v))|cells
        if regs is None or bin(v^vis).count('1')>1:
            regs=full(cells,a,P); stats[0]+=1
        elif v!=vis:
            d=v^vis; p=d.bit_length()-1; bit=d
            if v&d:
                hit=[r for r in regs if r&bit]
                if hit:
                    if LUT[ring_index(a,p,P)]:
                        regs=[r&~bit for r in regs]; stats[1]+=1
                    else:
                        R=hit[0]&~bit; regs=[r for r in regs if not r&bit]
                        rest=R&cells
                        while rest:
                            pc=flood(rest&-rest,a,P); regs.append(pc); rest&=~pc
                        stats[2]+=1
            else:
                if a&bit:
                    nb=((bit<<1)|(bit>>1)|((bit<<P)&M)|(bit>>P))&a
                    allp=0
                    for r in regs: allp|=r
                    hit=[r for r in regs if r&nb]
                    if hit:
                        merged=bit|(nb&~allp)
                        for r in hit: merged|=r
                        regs=[r for r in regs if not r&nb]+[merged]
                        stats[3]+=1
        vis=v
        ref=sorted(full(cells,a,P))
        assert sorted(regs)==ref,(seed,t)
    return stats


def main(boards=3000):
    tot = [0, 0, 0, 0]
    for s in range(boards):
        st = run(s)
        tot = [a + b for a, b in zip(tot, st)]
    return tot


if __name__ == "__main__":
    print("ok rebuild/simple/split/add", main(int(sys.argv[1]) if len(sys.argv) > 1 else 3000))
