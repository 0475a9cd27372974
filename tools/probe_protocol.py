import sys, os
sys.path[:0] = ["tests", "."]
import numpy as np, torch
from nimblephysics_amd import workloads, _native
lib = os.environ.get("NIMBLE_AMD_LIB", "product")
w = workloads.atlas_mesh_world(True)
B = 256
st, f = workloads.atlas_states(w, B, 1000)
d = torch.device("cuda:0")
dev = w.native()
cache = torch.zeros((B, dev.cache_doubles), dtype=torch.float64, device=d); cache[:, 0] = -1
snap = torch.zeros((B, dev.snapshot_doubles), dtype=torch.float64, device=d)
nxt = torch.empty((B, st.shape[1]), dtype=torch.float64, device=d)
import time
t0 = time.time()
dev.forward(torch.tensor(st, device=d), torch.tensor(f, device=d), cache, nxt, snap, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
sn = snap.cpu().numpy()
stat = sn[:, 5].astype(int)
print(lib, "forward s", round(time.time() - t0, 3), "protocol worlds", int(((stat & 64) != 0).sum()), "contact worlds", int((sn[:, 0] > 0).sum()),
      "deferred", int(((stat & 32) != 0).sum()))
