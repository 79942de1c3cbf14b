"""visionseg — MI355X-native Swin + Mask2Former training hot path.

Hand-written gfx950 HIP kernels (libvisionseg_hip.so, C ABI in include/visionseg.h)
for Swin window partition/attention, multi-scale deformable attention, the mask head
and masked cross-attention, surfaced to PyTorch as autograd ops (`visionseg.ops`),
plus the model, criterion, data-parallel trainer and the adapters the reference's
callers use (`train_template.train_maskdino`, `AISegmentationModel`).
"""
__version__ = "0.1.0"

import os as _os

# HIP graphs (Trainer(graphs=True)): ROCm's graph packet capture (kernel packets and
# kernel arguments of a graph exec recorded once at instantiation) replayed graphs with
# the wrong kernel arguments after another graph was captured or destroyed -- illegal
# memory accesses on MI355X (tools/graph_diag.py --variant recapture).  Plain per-node
# graph launches cost nothing measurable here (59.2 vs 59.0 ms/step).  The runtime reads
# the flag once, at HIP initialisation: import visionseg before touching the device.
import sys as _sys

_flag_before = _os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE")
_torch = _sys.modules.get("torch")
_hip_up_before = bool(_torch is not None and hasattr(_torch, "cuda") and _torch.cuda.is_initialized())
_os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
# False when HIP was already initialised (by the caller) before the flag was in place:
# Trainer(graphs=True) refuses to capture then
GRAPH_CAPTURE_SAFE = (_os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"] == "0"
                      and (not _hip_up_before or _flag_before == "0"))
