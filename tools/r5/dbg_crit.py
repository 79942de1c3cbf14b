"""Debug: the smoke() model's fp32 loss with the target labels sampled by the HIP mask
kernel vs grid_sample (criterion._MASK_SAMPLE_KERNEL), same weights / batch / RNG."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-instance-seg_amd")]
import torch  # noqa: E402

from oracle.detinit import det_init  # noqa: E402
from oracle.ref_model import RefConfig, RefMask2Former  # noqa: E402
from visionseg import criterion as CR  # noqa: E402
from visionseg import ops  # noqa: E402
from visionseg.data import synthetic_batch  # noqa: E402
from visionseg.model import M2FConfig, Mask2Former  # noqa: E402

cfg = M2FConfig(embed_dim=32, depths=(2, 2, 2, 2), num_heads=(1, 2, 4, 8), feature_size=64, mask_feature_size=64,
                hidden_dim=64, enc_ffn=128, dec_ffn=128, dec_heads=2, enc_layers=2, dec_layers=4, num_queries=10,
                train_num_points=256)
ref = RefMask2Former(RefConfig.from_dict(cfg.to_dict())).eval()
sd = det_init({k: v.shape for k, v in ref.state_dict().items()}, 1234)
m = Mask2Former(cfg)
m.load_state_dict(sd)
m = m.cuda()
imgs, ml, cl = synthetic_batch(2, 128, seed=0)
print("mask dtypes", [x.dtype for x in ml], [x.shape for x in ml], flush=True)
with torch.no_grad():
    masks, classes = m(imgs.cuda())
tg = CR.PaddedTargets.from_lists([x.cuda() for x in ml], [x.cuda() for x in cl])
print("tg", tg.masks.dtype, tg.masks.shape, tg.masks.is_contiguous(), int(tg.masks.sum()))
for flag in (True, False):
    CR._MASK_SAMPLE_KERNEL = flag
    torch.cuda.manual_seed(5)
    loss, parts = CR.SetCriterion(cfg)(masks, classes, [x.cuda() for x in ml], [x.cuda() for x in cl])
    print(flag, float(loss), {k: round(float(v), 4) for k, v in list(parts.items())[-3:]}, flush=True)
g = torch.rand(2, 64, 1, 2, device="cuda") * 2 - 1
CR._MASK_SAMPLE_KERNEL = True
a = CR._target_points(tg, g)
CR._MASK_SAMPLE_KERNEL = False
b = CR._target_points(tg, g)
print("target points max diff", float((a - b).abs().max()), a.shape, b.shape)
u8 = tg.masks.view(torch.uint8)
print("u8 unique", torch.unique(u8).tolist(), "bool->u8 via to", torch.unique(tg.masks.to(torch.uint8)).tolist())
rnd = torch.rand(2, 3, 128, 128, device="cuda") > 0.7
print("rand-bool u8 unique", torch.unique(rnd.view(torch.uint8)).tolist())
a = ops.point_sample_masks(tg.masks.view(6, 128, 128), g.squeeze(2), grid_space=True, sets_per_coord=3)
import torch.nn.functional as F
b = F.grid_sample(tg.masks.float(), g, align_corners=False).squeeze(3).view(6, 64)
print("direct", float((a - b).abs().max()), a.max().item(), b.max().item())
c = ops.point_sample_masks(tg.masks.view(6, 128, 128).clone(), g.squeeze(2).contiguous(), grid_space=True, sets_per_coord=3)
print("clone", float((c - b).abs().max()))
