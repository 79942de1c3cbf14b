"""Keyed random point draws for criterion parity (test infrastructure).

HF's criterion (and oracle.ref_model.RefCriterion) draws its matcher and loss points
per decoder step and per image with `torch.rand`, in call order; the product criterion
(visionseg.criterion.SetCriterion) batches all steps, images and targets into a few
draws.  The same points can only reach both when the draws are keyed by what they are
FOR: (image) for the matcher's uniform points (the product shares one set per image
across the decoder steps), (step, image, target) for the importance-sampling
candidates ("over") and the uniform remainder ("rand").  Both criteria accept such a
`point_source`.
"""
from __future__ import annotations

import zlib

import torch


class KeyedDraws:
    def __init__(self, max_images: int, max_targets: int, seed: int = 0):
        self.B, self.K, self.seed = max_images, max_targets, seed
        self._cache = {}

    def _table(self, key, shape):
        t = self._cache.get(key)
        if t is None:
            g = torch.Generator().manual_seed(self.seed * 1000003 + zlib.crc32(repr(key).encode()))
            t = self._cache[key] = torch.rand(shape, generator=g)
        return t

    def match_points(self, B, P, device=None):
        assert B <= self.B
        return self._table(("match", P), (self.B, P, 2))[:B].to(device if device is not None else "cpu")

    def loss_points(self, S, B, Kc, n, kind, device=None):
        assert B <= self.B and Kc <= self.K and kind in ("over", "rand")
        t = self._table((kind, S, n), (S, self.B, self.K, n, 2))[:, :B, :Kc]
        return t.to(device if device is not None else "cpu")
