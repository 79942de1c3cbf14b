"""visionseg — MI355X-native Swin + Mask2Former training hot path.

Hand-written gfx950 HIP kernels (libvisionseg_hip.so, C ABI in include/visionseg.h)
for Swin window partition/attention, multi-scale deformable attention, the mask head
and masked cross-attention, surfaced to PyTorch as autograd ops (`visionseg.ops`),
plus the model, criterion, data-parallel trainer and the adapters the reference's
callers use (`train_template.train_maskdino`, `AISegmentationModel`).
"""
__version__ = "0.1.0"
