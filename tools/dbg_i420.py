import sys, numpy as np, torch
sys.path.insert(0,'.'); sys.path.insert(0,'oracle')
import __graft_entry__ as g; evam=g.import_package(); import oracle as O
c=O.COracle()
rng=np.random.default_rng(0)
def run(f, DW, DH, rois=None):
    img=evam.Image.from_host(f.fourcc,f.width,f.height,f.planes,device='cuda:0')
    n = len(rois) if rois else 1
    out=torch.zeros((n,3,DH,DW),dtype=torch.uint8,device='cuda:0')
    pp=evam.HipPreProcessor(0); pp.convert([img],out, rois=[evam.Roi(*r) for r in rois] if rois else None); torch.cuda.synchronize()
    got=out.cpu().numpy(); ref=np.zeros_like(got)
    for i,r in enumerate(rois or [(0,0,0,0,0)]):
        c.preprocess_item(f,r[1:],ref,i)
    return got, ref
W,H=64,48
f=O.random_frame(rng,O.I420,W,H)
f.planes[1][:]=128; f.planes[2][:]=128
got,ref=run(f,512,512); print('chroma const: mism', int((got!=ref).sum()))
f=O.random_frame(rng,O.I420,W,H)
f.planes[0][:]=128
got,ref=run(f,512,512); bad=np.argwhere(got[0]!=ref[0]); print('Y const: mism', len(bad))
rows=sorted(set(bad[:,1].tolist())); print(' bad rows', rows[:40], len(rows)); cols=sorted(set(bad[:,2].tolist())); print(' bad cols', cols[:40], len(cols))
# BGR ROI case
f=O.random_frame(rng,O.BGR,320,240)
for roi in [(0,1,1,1,1),(0,5,7,9,11),(0,100,100,3,3),(0,0,0,320,240),(0,10,10,100,80)]:
    got,ref=run(f,72,72,[roi]); bad=np.argwhere(got[0]!=ref[0])
    print('BGR roi',roi,'mism',len(bad), 'rows', sorted(set(bad[:,1].tolist()))[:20])
for fmt in (O.NV12,O.BGRX):
  f=O.random_frame(rng,fmt,320,240)
  for roi in [(0,1,1,1,1),(0,5,7,9,11),(0,100,100,3,3)]:
    got,ref=run(f,72,72,[roi]); bad=np.argwhere(got[0]!=ref[0])
    print(hex(fmt),'roi',roi,'mism',len(bad), 'rows', sorted(set(bad[:,1].tolist()))[:20])
