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


class ForcedDecisions(KeyedDraws):
    """KeyedDraws that also carries the DECISIONS of one criterion run into later runs:
    the Hungarian matching of every decoder step and the importance-sampling choice
    (top-k most uncertain of the oversampled points) of every (step, image, target).

    The first oracle run records them (`replay` False); with `replay` True the oracle
    (RefCriterion hooks `forced_match` / `select`) and the product
    (SetCriterion hooks `forced_assign` / `select`) take the recorded ones.  At bf16
    resolution a near-tie flips a matching or swaps a point at the top-k boundary; those
    are decisions, not arithmetic, and forcing them leaves only the arithmetic to compare
    (as the decoder's attention masks are forced through `mask_override`)."""

    def __init__(self, max_images: int, max_targets: int, seed: int = 0):
        super().__init__(max_images, max_targets, seed)
        self.replay = False
        self.matches = {}                # step -> [(query idx, target idx)] per image
        self.top = {}                    # (step, image, target) -> selected candidate indices

    # oracle: RefCriterion.single
    def forced_match(self, step, idx):
        if not self.replay:
            self.matches[int(step)] = [(a.clone(), b.clone()) for a, b in idx]
            return idx
        return self.matches[int(step)]

    # product: SetCriterion.__call__, int32 [S, B, Kc] query per target (-1 = none)
    def forced_assign(self, assign):
        assert self.replay
        S, B, Kc = assign.shape
        out = torch.full((S, B, Kc), -1, dtype=torch.int32)
        for s in range(S):
            for i, (a, b) in enumerate(self.matches[s]):
                out[s, i, b] = a.to(torch.int32)
        return out.to(assign.device)

    def select(self, unc, nu, step, img, tgt):
        own = torch.topk(unc, k=nu, dim=1)[1]
        keys = list(zip(step.tolist(), img.tolist(), tgt.tolist()))
        if not self.replay:
            for r, k in enumerate(keys):
                self.top[k] = own[r].cpu()
            return own
        rows = [r for r, k in enumerate(keys) if k in self.top]     # padded slots keep their own
        if rows:
            own = own.clone()
            own[torch.tensor(rows, device=own.device)] = torch.stack([self.top[keys[r]] for r in rows]).to(own.device)
        return own
