import numpy as np, sys
a=np.load(sys.argv[1]); b=np.load(sys.argv[2])
for k in a.files:
    x,y=a[k],b[k]
    d=~((x==y)|(np.isnan(x)&np.isnan(y)))
    nt = int(d.reshape(d.shape[0],-1).any(1).sum()) if d.ndim>1 else -1
    rel = float(np.nanmax(np.abs(x-y))/max(1e-30,np.nanmax(np.abs(x)))) if x.dtype.kind=='f' else 0
    print(k, x.shape, 'differ elems', int(d.sum()), 'traj', nt, 'maxrel', rel)
