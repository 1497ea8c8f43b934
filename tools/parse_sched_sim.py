"""Discrete-event model of the H.264 parse pool on the C3 stream (I P B B P B B ..., 60 pictures): 16
workers, the lookahead dispatching a picture every 0.08 ms, P ~4.6 ms / B ~4.8 ms / I ~6 ms of parse (the
r96 timeline), each B picture waiting for its anchor, then in-order submission (0.14 ms) and a device
taking 0.27 ms per picture.  Prints the mean parse end and device end over 20 jittered runs for windows
W of h264_async.c pick_job (anchors within W jobs of the oldest first; 0 = oldest first).
Usage: python3 tools/parse_sched_sim.py"""
import heapq, random
def sim(W, workers=16, n=60, seed=0, gpu=0.27, sub=0.14, jitter=0.1):
    rnd=random.Random(seed)
    typ=[]; dep=[]
    for k in range(n):
        if k==0: typ.append(2); dep.append(None)
        elif k%3==1: typ.append(0); dep.append(None)
        else: typ.append(1); dep.append(k-1 if k%3==2 else k-2)
    dur=[(6.0 if t==2 else 4.6 if t==0 else 4.8)*(1+rnd.uniform(-jitter,jitter)) for t in typ]
    disp=[0.76+0.08*k for k in range(n)]
    done=[None]*n; taken=[False]*n
    t=0.0; free=workers; ev=[]  # (time, job)
    while True:
        # assign
        while free>0:
            oldest=next((k for k in range(n) if not taken[k] and disp[k]<=t), None)
            if oldest is None: break
            cands=[k for k in range(n) if not taken[k] and disp[k]<=t and (dep[k] is None or (done[dep[k]] is not None and done[dep[k]]<=t))]
            if not cands: break
            pick=None
            if W>0:
                refs=[k for k in cands if typ[k]!=1 and k<oldest+W]
                if refs: pick=refs[0]
            if pick is None: pick=cands[0]
            taken[pick]=True; free-=1; heapq.heappush(ev,(t+dur[pick],pick))
        nxt=[e[0] for e in ev]+[d for k,d in enumerate(disp) if not taken[k] and d>t]
        if not nxt: break
        tn=min(nxt)
        while ev and ev[0][0]<=tn:
            te,k=heapq.heappop(ev); done[k]=te; free+=1
        t=tn
    pend=max(done)
    s=0; g=0
    for k in range(n):
        s=max(s,done[k])+sub
        g=max(g,s)+gpu
    return pend, g
if __name__ == '__main__':
  for W in (0,2,4,6,8,10,12,16,20,24,32,64):
    r=[sim(W,seed=s) for s in range(20)]
    print(W, 'parse end %.2f  gpu end %.2f'%(sum(x[0] for x in r)/20, sum(x[1] for x in r)/20))
