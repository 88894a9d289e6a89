import sys, time
sys.path.insert(0, "/root/repo/3d-matching_amd")
import numpy as np, torch
from m3d import prep, synth
from m3d.core import Cloud, to_device
v, _ = synth.surface_mesh(300, 600, seed=1)
pts = v.astype(np.float32).astype(np.float64)
for rep in range(3):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    c = Cloud(pts); torch.cuda.synchronize(); t1 = time.perf_counter()
    prep.estimate_normals(c, 0.6, 30); t2 = time.perf_counter()
    prep.estimate_normals(c, 0.6, 30); t3 = time.perf_counter()
    x = torch.empty((len(pts), 3), dtype=torch.float64, device="cuda"); torch.cuda.synchronize()
    t4 = time.perf_counter(); x.cpu(); t5 = time.perf_counter()
    print(f"cloud {1e3*(t1-t0):.2f} normals(first, grids built) {1e3*(t2-t1):.2f} normals(grids cached) {1e3*(t3-t2):.2f} d2h 4.3MB {1e3*(t5-t4):.2f}")
