#!/usr/bin/env python3
"""Lock-step cost of the W = 1 rule audit's flood fills (audit_r in sparc_rules.hpp) under ways of
assigning a tile's env-step audits to the lanes of a wave (k_rollout1r): random walks with pops and
resets on 7 x 7 lattices with gaps, every audit's regions flooded with the kernel's dilation, and a
wave-audit costed as the sum over region index k of the slowest lane's k-th flood.  Prints the
useful iterations per lane-audit and the lock-step iterations per wave-audit of: lanes on 64 envs
at one step (the round-5 kernel), groupings by the previous cost, env-major blocks and the
env-major consecutive order k_rollout1r now uses (`consec`).  CPU only (a few minutes).
--pool: the same count on the bench's c3r pool (bench.make_pool: its gaps, starts and targets)
with env-like walks (random actions, traceback pops, the target ends the episode and the env
moves on to the next puzzle): round-5 order 37.8, env-major 25.5, useful 10.3 per lane-audit.

    python tools/audit_lockstep_sim.py [--pool]
"""
import os
import random
import sys
M=(1<<64)-1
def flood_iters(seed,a,P):
    r=seed; it=0
    while True:
        it+=1
        up=((((a+r)&M)^a)&a)|r
        nx=(up|(r>>1)|((r<<P)&M)|(r>>P))&a
        if nx==r: return r,it
        r=nx
def regions(cells,a,P):
    rem=cells; its=[]
    while rem:
        R,it=flood_iters(rem&-rem,a,P); its.append(it); rem&=~(R&cells)
    return its
rnd=random.Random(1)
X=Y=7;P=8
lattice=0;cells=0
for x in range(X):
    for y in range(Y):
        b=x*P+y
        if x%2==1 and y%2==1: cells|=1<<b
        else: lattice|=1<<b
def mkpuz():
    gaps=0
    for x in range(X):
        for y in range(Y):
            if (x+y)%2==1 and rnd.random()<0.1: gaps|=1<<(x*P+y)
    return gaps
puz=[mkpuz() for _ in range(256)]
pts=[(x,y) for x in range(0,X,2) for y in range(0,Y,2)]
class Env:
    def __init__(s): s.reset()
    def reset(s):
        s.g=rnd.choice(puz); s.path=[rnd.choice(pts)]; s.steps=0
    def step(s):
        s.steps+=1
        a=rnd.randrange(4)
        x,y=s.path[-1]; dx,dy=[(1,0),(-1,0),(0,1),(0,-1)][a]
        nx,ny=x+dx,y+dy
        if len(s.path)>1 and (nx,ny)==s.path[-2]: s.path.pop()
        elif 0<=nx<X and 0<=ny<Y and not(nx%2 and ny%2) and (nx,ny) not in s.path and not (s.g>>(nx*P+ny))&1: s.path.append((nx,ny))
        if s.steps>=40 or rnd.random()<0.02: s.reset()
    def cost(s):
        v=0
        for (x,y) in s.path: v|=1<<(x*P+y)
        a=(lattice&~(s.g|v))|cells
        return regions(cells,a,P)
def flat(jobs):
    # one loop over dilations: a lane that converges finishes its region and seeds the next in the
    # same iteration; cost = the longest lane's total, and the finish block runs in every
    # iteration where some lane ends a region
    ends=set()
    for j in jobs:
        t=0
        for it in j:
            t+=it; ends.add(t)
    return max(sum(j) for j in jobs), len(ends)
def lockstep(jobs):
    # jobs: list of region-iteration lists; cost = sum over k of max iters, + per-region overhead
    K=max(len(j) for j in jobs)
    it=sum(max((j[k] if k<len(j) else 0) for j in jobs) for k in range(K))
    return it,K


def demo():
    N=1280; envs=[Env() for _ in range(N)]
    RT=10; A=5
    tot={'fixed':[0,0],'prev':[0,0],'ideal':[0,0]}; useful=0
    prev=[sum(e.cost()) for e in envs]
    for tile in range(30):
        costs=[[None]*N for _ in range(RT)]
        for j in range(RT):
            for i,e in enumerate(envs):
                e.step(); costs[j][i]=e.cost()
        useful+=sum(sum(c) for row in costs for c in row)
        # fixed: groups of 64 envs, each step
        for j in range(RT):
            for g in range(N//64):
                it,K=lockstep(costs[j][g*64:(g+1)*64]); tot['fixed'][0]+=it; tot['fixed'][1]+=K
        jobs=[(j,i) for j in range(RT) for i in range(N)]
        # prev-cost sorted: key = env's last known cost (before the tile)
        key=lambda ji: prev[ji[1]]
        for name,kf in (('prev',key),('ideal',lambda ji: (len(costs[ji[0]][ji[1]]),sum(costs[ji[0]][ji[1]])))):
            js=sorted(jobs,key=kf)
            for b in range(0,len(js),64):
                it,K=lockstep([costs[j][i] for (j,i) in js[b:b+64]]); tot[name][0]+=it; tot[name][1]+=K
        prev=[sum(costs[RT-1][i]) for i in range(N)]
    nj=30*RT*N/64
    print("useful iters per lane-job %.2f"%(useful/(30*RT*N)))
    for k,v in tot.items(): print(k, "lockstep iters per wave-job %.2f, regions %.2f"%(v[0]/nj, v[1]/nj))

    # env-major assignments
    def run_assign(RT, A, E=128, tiles=20, sort=False, seed=2):
        global rnd
        rnd=random.Random(seed)
        envs=[Env() for _ in range(E)]
        L=RT//A; waves=A*E//64
        total=0; useful=0; prevk=[(0,0)]*E
        for t in range(tiles):
            costs=[[None]*E for _ in range(RT)]
            for j in range(RT):
                for i,e in enumerate(envs):
                    e.step(); costs[j][i]=e.cost()
            useful+=sum(sum(c) for row in costs for c in row)
            order=sorted(range(E),key=lambda i: prevk[i]) if sort else list(range(E))
            for w in range(waves):
                for m in range(L):
                    jobs=[]
                    for l in range(64):
                        J=(w*64+l)*L+m; env=order[J//RT]; step=J%RT
                        jobs.append(costs[step][env])
                    total+=lockstep(jobs)[0]
            prevk=[(len(costs[RT-1][i]),sum(costs[RT-1][i])) for i in range(E)]
        nj=tiles*RT*E/64
        return total/nj, useful/(tiles*RT*E)
    def run_fixed(RT, A, E=128, tiles=20, seed=2):
        global rnd
        rnd=random.Random(seed)
        envs=[Env() for _ in range(E)]
        total=0
        for t in range(tiles):
            costs=[[None]*E for _ in range(RT)]
            for j in range(RT):
                for i,e in enumerate(envs):
                    e.step(); costs[j][i]=e.cost()
            for j in range(RT):
                for g in range(E//64):
                    total+=lockstep(costs[j][g*64:(g+1)*64])[0]
        return total/(tiles*RT*E/64)
    print("fixed <2,5,10>", "%.2f"%run_fixed(10,5))
    for RT,A in ((10,5),(20,5),(30,5),(40,5),(20,10)):
        print("env-major RT=%d A=%d: %.2f (useful %.2f)"%((RT,A)+run_assign(RT,A)), " sorted: %.2f"%run_assign(RT,A,sort=True)[0])
    def run_consec(RT, A, E=128, tiles=20, sort=False, seed=2):
        global rnd
        rnd=random.Random(seed)
        envs=[Env() for _ in range(E)]
        waves=A*E//64; L=RT//A
        total=0; prevk=[(0,0)]*E
        for t in range(tiles):
            costs=[[None]*E for _ in range(RT)]
            for j in range(RT):
                for i,e in enumerate(envs):
                    e.step(); costs[j][i]=e.cost()
            order=sorted(range(E),key=lambda i: prevk[i]) if sort else list(range(E))
            for w in range(waves):
                for m in range(L):
                    jobs=[]
                    for l in range(64):
                        J=w*64+l+m*waves*64; env=order[J//RT]; step=J%RT
                        jobs.append(costs[step][env])
                    total+=lockstep(jobs)[0]
            prevk=[(len(costs[RT-1][i]),sum(costs[RT-1][i])) for i in range(E)]
        return total/(tiles*RT*E/64)
    for RT,A in ((10,5),(12,4),(20,10),(16,8)):
        print("consec RT=%d A=%d: %.2f sorted %.2f"%(RT,A,run_consec(RT,A),run_consec(RT,A,sort=True)))


# ---- the bench's c3r pool (bench.make_pool: real gaps, starts and targets) and env-like walks:
# uniform random actions, a move onto path[-2] pops (traceback), illegal moves do nothing, the
# target ends the episode and the env moves to the next puzzle (next-step autoreset, pid + 1)
def pool_mode(envs=1280, tiles=20, RT=10, A=5, seed=3):
    sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "sparc-gym_amd")]
    import bench
    sizes, full, _, _ = bench.CONFIGS["c3r"]
    pool = bench.make_pool(1024, sizes, full, workers=1)
    P = 8
    puz = []
    for p in pool:
        X, Y = int(p["x_size"]), int(p["y_size"])
        g = p["obs_array"]["gaps"]
        cellsb = latb = gapb = 0
        for x in range(X):
            for y in range(Y):
                b = 1 << (x * P + y)
                if x % 2 == 1 and y % 2 == 1:
                    cellsb |= b
                else:
                    latb |= b
                    if g[x][y]:
                        gapb |= b
        puz.append((X, Y, cellsb, latb, gapb, tuple(p["start_location"]), tuple(p["target_location"])))
    r = random.Random(seed)

    class E:
        def __init__(s, q):
            s.q = q
            s.reset()

        def reset(s):
            X, Y, c, l, g, st, tg = puz[s.q]
            s.path = [st]

        def step(s):
            X, Y, c, l, g, st, tg = puz[s.q]
            if s.path[-1] == tg:   # autoreset after the terminating step
                s.q = (s.q + 1) % len(puz)
                s.reset()
                return
            x, y = s.path[-1]
            dx, dy = ((0, -1), (1, 0), (0, 1), (-1, 0))[r.randrange(4)]
            nx, ny = x + dx, y + dy
            if len(s.path) > 1 and (nx, ny) == s.path[-2]:
                s.path.pop()
            elif 0 <= nx < X and 0 <= ny < Y and (l >> (nx * P + ny)) & 1 and not (g >> (nx * P + ny)) & 1 \
                    and (nx, ny) not in s.path:
                s.path.append((nx, ny))

        def cost(s):
            X, Y, c, l, g, st, tg = puz[s.q]
            v = 0
            for (x, y) in s.path:
                v |= 1 << (x * P + y)
            return regions(c, (l & ~(g | v)) | c, P)

    envs_ = [E((i * 2654435761) % len(puz)) for i in range(envs)]
    for _ in range(300):            # off the reset states
        for e in envs_:
            e.step()
    fixed = consec = 0
    useful = 0
    fl_it = fl_fin = ns_reg = 0
    for t in range(tiles):
        costs = [[None] * envs for _ in range(RT)]
        for j in range(RT):
            for i, e in enumerate(envs_):
                e.step()
                costs[j][i] = e.cost()
        useful += sum(sum(c) for row in costs for c in row)
        for j in range(RT):
            for g in range(envs // 64):
                fixed += lockstep(costs[j][g * 64:(g + 1) * 64])[0]
        for w0 in range(0, envs * RT, 64):      # env-major: 64 consecutive (env, step) jobs
            jobs = [costs[J % RT][J // RT] for J in range(w0, w0 + 64)]
            it, K = lockstep(jobs)
            consec += it
            ns_reg += K
            a, b = flat(jobs)
            fl_it += a
            fl_fin += b
    nj = tiles * RT * envs / 64
    print("c3r pool: useful iters per lane-audit %.2f; lock-step per wave-audit: lanes on 64 envs at one "
          "step %.2f, env-major %.2f" % (useful / (tiles * RT * envs), fixed / nj, consec / nj))
    print("env-major nested: %.2f iterations + %.2f region finishes per wave-audit; flattened: %.2f "
          "iterations, %.2f of them with a region finish" % (consec / nj, ns_reg / nj, fl_it / nj, fl_fin / nj))


if __name__ == "__main__":
    if "--pool" in sys.argv:
        pool_mode()
    else:
        demo()
