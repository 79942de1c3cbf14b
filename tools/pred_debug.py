"""Predictor graph-replay vs eager, per shape: max score difference (debug aid)."""
import os
import sys
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vision-instance-seg_amd")]
import numpy as np
import torch
import visionseg  # noqa: F401
from visionseg.inference import Predictor
from visionseg.model import M2FConfig, Mask2Former

print("DEBUG_CLR_GRAPH_PACKET_CAPTURE =", os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE"))
if len(sys.argv) > 2 and sys.argv[2] == "det":
    torch.backends.cudnn.deterministic = True
print("benchmark / deterministic set by args:", sys.argv[1:])
cfg = M2FConfig.preset("swin_t")
m = Mask2Former(cfg).init_weights(0)
maxg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
pg = Predictor(m, device="cuda:0", min_size=256, max_size=320, graphs=True, max_graphs=maxg)
pe = Predictor(m, device="cuda:0", min_size=256, max_size=320, graphs=False)
pe2 = Predictor(m, device="cuda:0", min_size=256, max_size=320, graphs=False)
rng = np.random.default_rng(0)
for shape in ((200, 260), (256, 256), (300, 180), (200, 260)) * int(os.environ.get("PASSES", "1")):
    img = rng.integers(0, 256, (*shape, 3)).astype(np.uint8)
    a, b, c = pg(img).pred_instances, pe(img).pred_instances, pe2(img).pred_instances
    print(shape, "graph-eager", float((a.scores - b.scores).abs().max()), "eager-eager", float((c.scores - b.scores).abs().max()),
          "masks eq", bool(torch.equal(a.masks, b.masks)))
