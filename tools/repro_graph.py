"""Repro helper: the eager loop of tests/test_graph_gpu.py (dropout 0.2, H=64, B=4) under given
pis_tune settings, e.g. python tools/repro_graph.py 26=1 27=0"""
import sys
import torch
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from physics_informed_image_segmentation_amd import AdamW, DiceBCEPDELoss, UNet, _hip
from physics_informed_image_segmentation_amd.dataset import disc_sample

for kv in sys.argv[1:]:
    k, v = kv.split("=")
    _hip.lib().pis_tune(int(k), int(v))
H, B, dropout = 64, 4, float(__import__("os").environ.get("DROPOUT", "0.2"))
g = torch.Generator().manual_seed(5)
imgs, masks = zip(*[disc_sample(H, H, g) for _ in range(B)])
x, t = torch.stack(imgs).cuda(), torch.stack(masks).cuda()
torch.manual_seed(42)
m = UNet(1, 1, 64, dropout=dropout).cuda().train()
opt = AdamW(m.parameters(), lr=1e-3, weight_decay=1e-5)
crit = DiceBCEPDELoss(pde_weight=1e-2, phase_field_weight=1e-2, diffusion_coeff=5.0, epsilon=0.05)
torch.cuda.manual_seed(11)
for i in range(5):
    opt.zero_grad(set_to_none=True)
    loss = crit(m(x), t)
    loss.backward()
    opt.step()
    torch.cuda.synchronize()
    print(i, loss.item(), flush=True)
print("ok", sys.argv[1:])
