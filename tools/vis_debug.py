import sys, numpy as np, torch
sys.path[:0]=["/root/repo","/root/repo/oracle","/root/repo/tests"]
import oracle, soc_real_time_renderer_amd as soc
from soc_real_time_renderer_amd import raster, multi_gpu
from soc_real_time_renderer_amd.scene import sponza_mesh
from helpers import globals_for
W,H,rank=480,270,3
g=globals_for(W,H,camera=multi_gpu.camera_for_rank(rank))
m=sponza_mesh.build()
hm=raster.MeshBuffers(m["positions"],m["normals"],m["uvs"],m["indices"],m["materials"])
dm=raster.MeshBuffers.from_numpy(m["positions"],m["normals"],m["uvs"],m["indices"],m["materials"])
vp=np.ctypeslib.as_array(g.camera_projection_view_matrix)
ref=np.zeros((H,W),np.uint64); oracle.raster_visibility(hm,vp,raster.CULL_FRONT,ref)
ws=dm.workspace(); vis=torch.zeros((H,W),dtype=torch.int64,device="cuda")
raster.raster_visibility(dm,vp,raster.CULL_FRONT,vis,ws); torch.cuda.synchronize()
got=vis.cpu().numpy().view(np.uint64)
bad=np.argwhere(got!=ref)
print("mismatch", len(bad))
for y,x in bad[:10]:
    for nm,v in (("gpu",got[y,x]),("cpu",ref[y,x])):
        low=int(v)&0xffffffff; tri=-1 if low==0xffffffff else 0xfffffffe-low
        z=np.uint32(int(v)>>32).view(np.float32)
        print(y,x,nm,tri,z, m["materials"][tri] if tri>=0 else None, m["indices"][tri] if tri>=0 else None)
# single-triangle rasters of the two candidates
for tri in (189587, 186530):
    idx = m["indices"][tri:tri + 1].copy()
    mats = m["materials"][tri:tri + 1].copy()
    h1 = raster.MeshBuffers(m["positions"], m["normals"], m["uvs"], idx, mats)
    d1 = raster.MeshBuffers.from_numpy(m["positions"], m["normals"], m["uvs"], idx, mats)
    r1 = np.zeros((H, W), np.uint64); oracle.raster_visibility(h1, vp, raster.CULL_FRONT, r1)
    v1 = torch.zeros((H, W), dtype=torch.int64, device="cuda")
    raster.raster_visibility(d1, vp, raster.CULL_FRONT, v1, d1.workspace()); torch.cuda.synchronize()
    g1 = v1.cpu().numpy().view(np.uint64)
    cov_c = (r1 & np.uint64(0xffffffff)) != np.uint64(0xffffffff)
    cov_g = (g1 & np.uint64(0xffffffff)) != np.uint64(0xffffffff)
    print("tri", tri, "cpu covers", int(cov_c.sum()), "gpu covers", int(cov_g.sum()), "differ", int((cov_c != cov_g).sum()),
          "depth differ", int(((r1 >> np.uint64(32)) != (g1 >> np.uint64(32)))[cov_c & cov_g].sum()),
          "at pixel cpu", cov_c[190, 240], "gpu", cov_g[190, 240])
    P = m["positions"][m["indices"][tri]]
    clip = np.c_[P, np.ones(3)].astype(np.float64) @ vp.reshape(4, 4).astype(np.float64)
    print("  clip", clip.tolist())
