"""fp8 (MX) window attention forward on one small case: NaN census per (window, head,
query tile) and the error vs the CPU emulation (tests/test_gpu_fp8.py)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vision-instance-seg_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import test_gpu_fp8 as T  # noqa: E402
from visionseg import ops  # noqa: E402

for dbg in ("0", "1", "2", "4", "7"):
  os.environ["VS_FP8_DBG"] = dbg
  print("VS_FP8_DBG", dbg)
  for cfg in (T.CASES[4], T.CASES[0]):
      qkv, table, _ = T._inputs(cfg, 11)
      geo = (cfg["heads"], cfg["ws"], cfg["shift"], cfg["nWh"], cfg["nWw"])
      with torch.no_grad():
          out = ops.window_attention(qkv.cuda(), table.cuda(), *geo, fp8=True).float().cpu()
          outb = ops.window_attention(qkv.cuda(), table.cuda(), *geo, fp8=False).float().cpu()
      emu, _ = T.emulate_fwd(qkv, table, *geo)
      N = cfg["ws"] ** 2
      o = out.view(out.shape[0], N, cfg["heads"], 32)
      nanmask = torch.isnan(o)
      print(f"ws {cfg['ws']}: NaN fraction {float(nanmask.float().mean()):.3f}; NaN per query tile",
            [float(nanmask[:, 32 * t:32 * t + 32].float().mean()) for t in range((N + 31) // 32)],
            "per channel half", [float(nanmask[..., 16 * i:16 * i + 16].float().mean()) for i in range(2)])
      ok = ~torch.isnan(out)
      if ok.any():
          print("  finite entries vs emulation max", float((out[ok] - emu[ok]).abs().max()), "vs bf16 path max",
                float((out[ok] - outb[ok]).abs().max()), "scale", float(outb.abs().max()))
      print("  sample fp8", out[0, :3, :6].tolist())
      print("  sample emu", emu[0, :3, :6].tolist())
