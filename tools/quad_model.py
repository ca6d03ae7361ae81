import numpy as np
def half_cleaner_cascade(x):
    x=x.copy(); n=len(x); s=n//2
    while s>=1:
        for i in range(n):
            if (i & s)==0:
                a,b=x[i],x[i+s]; x[i],x[i+s]=min(a,b),max(a,b)
        s//=2
    return x
def quad(r):
    lanes=[r[128*h:128*h+128].astype(np.float32) for h in range(4)]
    sgn0=[1,-1,-1,1]
    s=[np.sort(np.float32(sgn0[h])*lanes[h]) for h in range(4)]
    s=[np.minimum(s[h],-s[h^1]) for h in range(4)]
    for h in (1,3): s[h]=-s[h]
    s=[half_cleaner_cascade(x) for x in s]
    s=[np.minimum(s[h],-s[h^2]) for h in range(4)]
    for h in (1,3): s[h]=-s[h]
    s=[np.minimum(s[h],-s[h^1]) for h in range(4)]
    for h in (1,3): s[h]=-s[h]
    s=[half_cleaner_cascade(x) for x in s]
    z=np.concatenate([s[0], s[1], -s[3][::-1], -s[2][::-1]])
    return z
rng=np.random.default_rng(0)
for t in range(20):
    r=rng.standard_normal(512).astype(np.float32)
    if t%3==0: r=rng.integers(-3,4,512).astype(np.float32)
    if t%5==0: r[rng.integers(0,512,7)]=np.inf; r[rng.integers(0,512,5)]=-np.inf
    z=quad(r)
    assert np.array_equal(z, np.sort(r)), t
print("quad model sorts: ok")
