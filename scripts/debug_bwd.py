"""Debug dump of the backward's workspace (bring-up only): runs one small case through the
C ABI with a caller-owned workspace and saves the intermediate arrays to an npz."""
import ctypes, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import custereomatching_amd as cm
from custereomatching_amd import _lib
from tests.golden.inputs import make_pair

H, W, k, D = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
layout = sys.argv[5]
out = sys.argv[6]
lay = _lib.LAYOUT_FULL if layout == "full" else _lib.LAYOUT_WINDOW
Dl = D if layout == "window" else 0
cam, proj = make_pair(H, W, max(D, 1), seed=31)
c = torch.from_numpy(cam).cuda(); p = torch.from_numpy(proj).cuda()
vol = cm.cost_volume_forward(c, p, Dl, k, layout, "fast")
g = torch.from_numpy(np.random.default_rng(7).uniform(-1, 1, tuple(vol.shape)).astype(np.float32)).cuda()
nb = _lib.workspace_bytes(H, W, k, lay, Dl, _lib.OP_BACKWARD)
ws = torch.zeros(nb, dtype=torch.uint8, device="cuda")
gc = torch.empty(H, W, device="cuda"); gp = torch.empty(H, W, device="cuda")
rc = _lib.lib.custma_backward(g.data_ptr(), vol.data_ptr(), c.data_ptr(), p.data_ptr(), 0, H, W, k, lay, Dl,
                              gc.data_ptr(), gp.data_ptr(), ws.data_ptr(), ws.numel(),
                              torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
print("rc", rc, _lib.lib.custma_last_error())
np.savez(out, ws=ws.cpu().numpy(), gc=gc.cpu().numpy(), gp=gp.cpu().numpy(), g=g.cpu().numpy(),
         vol=vol.cpu().numpy(), cam=cam, proj=proj)
